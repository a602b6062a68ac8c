// comm.hip -- the multi-GPU exchange behind the C ABI (included by
// engine.hip): SURVEY.md §8b's "later" mpcr_comm_init and §8e's two
// exchanges, so a host without torch.distributed (the C / cgo / JNI hosts of
// INTEGRATION.md) can shard candidates over the GPUs of a node:
//   * the global best of a sharded rollout (idx_min = argmin(cost_batch[-1]),
//     SBP/mjx_planner.py:395): every rank's rollout kernel leaves a packed
//     key ordered(cost) << 32 | global index whose UNSIGNED order is the
//     jnp.argmin order (NaN first, ties to the lowest index), so one RCCL
//     uint64 MIN all-reduce is the global argmin;
//   * the sharded CEM elites (compute_ellite_samples, SBP/mjx_planner.py:305-310):
//     each rank's local top-kl rows (xi | cost) are all-gathered rank-major and
//     the global top-k is selected from the gathered block -- the same
//     selection as manipulator_mujoco_amd/dist.py::gather_elites.
// RCCL is dlopen'ed at the first mpcr_comm_* call: librccl.so.1 resolves to
// the copy the process already holds (torch's) or ROCm's, so libmpcr.so has
// no link-time dependency on it and loads on hosts without RCCL.

#include <rccl/rccl.h>

namespace {

struct RcclApi {
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) =
      nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  bool ok = false;
};

const RcclApi* rccl_api() {
  static RcclApi api;
  static bool tried = false;
  if (tried) return api.ok ? &api : nullptr;
  tried = true;
  void* h = nullptr;
  for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
    if ((h = dlopen(name, RTLD_NOW | RTLD_GLOBAL))) break;
  if (!h) return nullptr;
  api.get_unique_id = reinterpret_cast<decltype(api.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
  api.comm_init_rank = reinterpret_cast<decltype(api.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
  api.comm_destroy = reinterpret_cast<decltype(api.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
  api.all_reduce = reinterpret_cast<decltype(api.all_reduce)>(dlsym(h, "ncclAllReduce"));
  api.all_gather = reinterpret_cast<decltype(api.all_gather)>(dlsym(h, "ncclAllGather"));
  api.error_string = reinterpret_cast<decltype(api.error_string)>(dlsym(h, "ncclGetErrorString"));
  api.ok = api.get_unique_id && api.comm_init_rank && api.comm_destroy && api.all_reduce && api.all_gather &&
           api.error_string;
  return api.ok ? &api : nullptr;
}

// (xi row | cost) of the local elites, rank-local rows for the all-gather
__global__ void pack_elites_kernel(const float* __restrict__ xi, const float* __restrict__ cost,
                                   const int* __restrict__ idx, int kl, int nv, float* __restrict__ out) {
  const int r = blockIdx.x;
  if (r >= kl) return;
  const int i = idx[r];
  for (int c = threadIdx.x; c <= nv; c += blockDim.x)
    out[(size_t)r * (nv + 1) + c] = c < nv ? xi[(size_t)i * nv + c] : cost[i];
}

}  // namespace

#define RCCLCHK(api, x)                                                                         \
  do {                                                                                          \
    const ncclResult_t r_ = (x);                                                                \
    if (r_ != ncclSuccess) return fail(MPCR_EHIP, "%s: %s", #x, (api)->error_string(r_));      \
  } while (0)

struct mpcr_comm {
  int rank = 0, nranks = 1, device = 0;
  ncclComm_t comm = nullptr;
  float* d_pack = nullptr;  // local elite rows (kl x (nv + 1)), grown on demand
  int* d_lidx = nullptr;    // local elite indices
  size_t pack_cap = 0;
  int lidx_cap = 0;
};

extern "C" int mpcr_comm_unique_id(unsigned char* id_out) {
  if (!id_out) return fail(MPCR_EINVAL, "null id");
  const RcclApi* api = rccl_api();
  if (!api) return fail(MPCR_EHIP, "RCCL (librccl.so.1) could not be loaded");
  ncclUniqueId id;
  RCCLCHK(api, api->get_unique_id(&id));
  std::memcpy(id_out, id.internal, MPCR_COMM_ID_BYTES);
  return MPCR_OK;
}

extern "C" int mpcr_comm_init(int rank, int nranks, const unsigned char* id, int device, mpcr_comm** out) {
  if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks) return fail(MPCR_EINVAL, "bad comm arguments");
  *out = nullptr;
  const RcclApi* api = rccl_api();
  if (!api) return fail(MPCR_EHIP, "RCCL (librccl.so.1) could not be loaded");
  HIPCHK(hipSetDevice(device));
  ncclUniqueId uid;
  std::memcpy(uid.internal, id, MPCR_COMM_ID_BYTES);
  mpcr_comm* c = new mpcr_comm;
  c->rank = rank; c->nranks = nranks; c->device = device;
  const ncclResult_t r = api->comm_init_rank(&c->comm, nranks, uid, rank);
  if (r != ncclSuccess) {
    delete c;
    return fail(MPCR_EHIP, "ncclCommInitRank: %s", api->error_string(r));
  }
  *out = c;
  return MPCR_OK;
}

extern "C" void mpcr_comm_free(mpcr_comm* c) {
  if (!c) return;
  const RcclApi* api = rccl_api();
  if (api && c->comm) api->comm_destroy(c->comm);
  (void)hipFree(c->d_pack);
  (void)hipFree(c->d_lidx);
  delete c;
}

extern "C" int mpcr_comm_allreduce_key(mpcr_comm* c, uint64_t* d_key, int count, void* stream) {
  if (!c || !d_key || count < 1) return fail(MPCR_EINVAL, "bad key all-reduce arguments");
  const RcclApi* api = rccl_api();
  HIPCHK(hipSetDevice(c->device));
  RCCLCHK(api, api->all_reduce(d_key, d_key, (size_t)count, ncclUint64, ncclMin, c->comm, (hipStream_t)stream));
  return MPCR_OK;
}

extern "C" int mpcr_comm_allgather(mpcr_comm* c, const float* d_send, float* d_recv, size_t count, void* stream) {
  if (!c || !d_send || !d_recv) return fail(MPCR_EINVAL, "bad all-gather arguments");
  const RcclApi* api = rccl_api();
  HIPCHK(hipSetDevice(c->device));
  RCCLCHK(api, api->all_gather(d_send, d_recv, count, ncclFloat32, c->comm, (hipStream_t)stream));
  return MPCR_OK;
}

extern "C" int mpcr_comm_gather_elites(mpcr_comm* c, const float* d_cost, const float* d_xi, int n, int nv, int k,
                                       float* d_rows, int* d_sel, void* stream) {
  if (!c || !d_cost || !d_xi || !d_rows || !d_sel || n < 1 || nv < 1 || k < 1)
    return fail(MPCR_EINVAL, "bad gather_elites arguments");
  const int kl = std::min(k, n);
  if ((long long)kl * c->nranks < k) return fail(MPCR_EINVAL, "k=%d elites need more than %d x %d candidates", k,
                                                 c->nranks, n);
  if (kl > TOPK_MAX || k > TOPK_MAX) return fail(MPCR_EINVAL, "k=%d above %d", k, TOPK_MAX);
  const RcclApi* api = rccl_api();
  HIPCHK(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  const size_t rowlen = (size_t)nv + 1, need = (size_t)kl * rowlen;
  if (need > c->pack_cap) {  // first call of a shape; graph capture replays a sized comm
    (void)hipFree(c->d_pack);
    c->d_pack = nullptr;
    HIPCHK(hipMalloc(&c->d_pack, sizeof(float) * need));
    c->pack_cap = need;
  }
  if (kl > c->lidx_cap) {
    (void)hipFree(c->d_lidx);
    c->d_lidx = nullptr;
    HIPCHK(hipMalloc(&c->d_lidx, sizeof(int) * kl));
    c->lidx_cap = kl;
  }
  hipLaunchKernelGGL(topk_kernel, dim3(1), dim3(1024), 0, st, d_cost, 1, n, kl, c->d_lidx);
  HIPCHK(hipGetLastError());
  hipLaunchKernelGGL(pack_elites_kernel, dim3(kl), dim3(64), 0, st, d_xi, d_cost, c->d_lidx, kl, nv, c->d_pack);
  HIPCHK(hipGetLastError());
  RCCLCHK(api, api->all_gather(c->d_pack, d_rows, need, ncclFloat32, c->comm, st));
  // global top-k over the gathered cost column: positions are rank-major and
  // each rank's rows are in (cost, index) order, so position ties are global
  // index ties (stable argsort order)
  hipLaunchKernelGGL(topk_kernel, dim3(1), dim3(1024), 0, st, d_rows + nv, (int)rowlen, c->nranks * kl, k, d_sel);
  HIPCHK(hipGetLastError());
  return MPCR_OK;
}
