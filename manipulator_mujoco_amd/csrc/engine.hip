// engine.hip — host side of the C ABI (include/mpcr.h): model blobs, the
// fp32 device model with its derived tables, engines, launches.
#include <hip/hip_runtime.h>
#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <limits>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mpcr.h"
#include "mpcr_device.h"

// kernels: the fused rollout is its own translation unit (rollout.hip, its
// launchers declared in rollout.h); cem.hip: the CEM distribution step
#include "rollout.h"

// extra dynamic LDS per narrow-kernel block (occupancy experiments only)
// horizon segments of dual-arm rollouts (rollout_launch): steps per segment
// (0 = one launch) and candidate groups on their own streams.  Measured
// (tools/seg_sweep_r04.sh; C4 shard 4096 x 100 / C5 rollout 8192 x 50, ms):
// one launch 50.6 / 48.5; 2 groups x 25 steps 47.8 / 47.4, x 13-10 46.7 /
// 45.8, x 7 46.3 / 45.0, x 5-3 46.4-46.6 / 45.1; 3 groups 47.3-49.5; 4
// groups 65-67 (more streams than the process's 4 hardware queues)
#ifndef MPCR_SEG_STEPS_DEFAULT
#define MPCR_SEG_STEPS_DEFAULT 7
#endif
#ifndef MPCR_SEG_GROUPS_DEFAULT
#define MPCR_SEG_GROUPS_DEFAULT 2
#endif
#define MPCR_SEG_MAXG 4
static int env_int_or(const char* name, int dflt) {
  const char* v = getenv(name);
  return v ? atoi(v) : dflt;
}
#ifndef MPCR_N_DYN_LDS
#define MPCR_N_DYN_LDS 0
#endif
#include "cem.hip"

namespace mpcr {
// argmin with NaN-first / first-index semantics over cost[i*stride]
__global__ void __launch_bounds__(256) argmin_kernel(const float* __restrict__ cost, int stride, int n, int base,
                                                     unsigned long long* key) {
  unsigned long long best = ~0ull;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float c = cost[(size_t)i * stride];
    const uint32_t u = __float_as_uint(c);
    const uint32_t k = isnan(c) ? 0u : ((u & 0x80000000u) ? ~u : (u | 0x80000000u));
    const unsigned long long k64 = ((unsigned long long)k << 32) | (uint32_t)(base + i);
    best = k64 < best ? k64 : best;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long other = __shfl_xor(best, o);
    best = other < best ? other : best;
  }
  if ((threadIdx.x & 63) == 0) atomicMin(key, best);
}

__global__ void fill_u64(unsigned long long* p, unsigned long long v) { *p = v; }

}  // namespace mpcr

using namespace mpcr;

struct mpcr_model {
  mpcr_model_t m;
};

struct mpcr_engine {
  int device = 0, max_n = 0, H = 0, nbasis = 0;
  mpcr_model_t host;
  DevModel dev;
  DevModel* d_model = nullptr;
  float* d_pdot = nullptr;
  // staging (host-pointer calls)
  float* d_in = nullptr;
  float* d_cost = nullptr;
  float* d_theta = nullptr;
  float* d_thetadot = nullptr;
  unsigned long long* d_key = nullptr;
  int* d_status = nullptr;
  int* d_idx = nullptr;
  float* d_slot_prev = nullptr;  // max_n x nslot (variants keeping cost_c history in HBM)
  float* d_jx = nullptr;         // max_n x (MAXEFC - JL) x LDJ: J rows past the LDS ones
  float* d_td = nullptr;         // (max_n + 1) x nctrl x H joint-velocity table (thetadot not requested)
  short* d_hints = nullptr;      // max_n x NHINT x 2 (dual-arm class): hull-climb starts
  unsigned* d_pace = nullptr;    // MPCR_PACE_SLOTS: the rollout kernel's per-wave-slot progress (pacing)
  float* d_mslab = nullptr;      // (max_n + 1) x NVW x LD: the dual-arm class's mass matrices
  // horizon segments of the dual-arm class (rollout_launch): steps per
  // segment, candidate groups and their streams / fork-join events
  float* d_seg = nullptr;        // max_n x SEG_STRIDE
  int seg_steps = 0, seg_groups = 1, seg_min_n = 0;
  hipStream_t seg_stream[MPCR_SEG_MAXG] = {};
  hipEvent_t seg_event[MPCR_SEG_MAXG + 1] = {};
  // convex hulls (dual-arm class)
  float4* d_hull_vert = nullptr;
  int2* d_hull_info = nullptr;
  float4* d_hull_adjv = nullptr;
  float4* d_hull_head = nullptr;
  float4* d_hull_lut = nullptr;
  // polygon faces (polyhedron-pair manifold)
  float4* d_face_plane = nullptr;
  int2* d_face_vinfo = nullptr;
  int* d_face_vert = nullptr;
  int2* d_vert_finfo = nullptr;
  int* d_vert_face = nullptr;
  int2* d_cone_cell = nullptr;
  int* d_cone_face = nullptr;
  bool wide = false;  // kernel variant: rollout_kernel<32, 32, 72, true>
};

// The narrow variant (16-wide solves, 16 bodies, 24 collision geoms, Euler,
// joint equalities only) covers the single-arm scenes; anything else runs the
// wide one (dual-arm class).
static bool needs_wide(const mpcr_model_t& m, const DevModel& d) {
  if (m.nv > 16 || d.nbody > 16 || d.ngeom > 24 || m.nq > MPCR_N_NQ || m.nu > 0 || d.has_spring ||
      m.integrator != MPCR_INT_EULER || m.cone != MPCR_CONE_PYRAMIDAL || m.nten > 0 || m.viscosity != 0)
    return true;
  for (int e = 0; e < m.neq; e++)
    if (m.eq_type[e] != MPCR_EQ_JOINT) return true;
  for (int p = 0; p < m.npair; p++)
    if (m.pair_func[p] == MPCR_COL_CONVEX || m.pair_func[p] == MPCR_COL_PLANE_CONVEX) return true;
  return false;
}

static thread_local std::string g_err;

static int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
static int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIPCHK(x)                                                                         \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) return fail(MPCR_EHIP, "%s: %s", #x, hipGetErrorString(e_));  \
  } while (0)

extern "C" const char* mpcr_last_error(void) { return g_err.c_str(); }
extern "C" int mpcr_abi_version(void) { return MPCR_ABI_VERSION; }

extern "C" int mpcr_device_arch(int device, char* buf, int buflen) {
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, device));
  snprintf(buf, buflen, "%s", prop.gcnArchName);
  return MPCR_OK;
}

// ---------------------------------------------------------------------------
// models

static int check_model(const mpcr_model_t& m) {
  if (m.magic != MPCR_MODEL_MAGIC) return fail(MPCR_EMODEL, "bad model magic 0x%x", m.magic);
  if (m.version != MPCR_MODEL_VERSION) return fail(MPCR_EMODEL, "model version %u != %d", m.version, MPCR_MODEL_VERSION);
  if (m.nbytes != sizeof(mpcr_model_t)) return fail(MPCR_EMODEL, "model size %u != %zu", m.nbytes, sizeof(mpcr_model_t));
  if (m.nbody > MPCR_MAX_BODY || m.njnt > MPCR_MAX_JNT || m.nv > MPCR_MAX_DOF || m.nq > MPCR_MAX_NQ ||
      m.ngeom > MPCR_MAX_GEOM || m.npair > MPCR_MAX_PAIR || m.neq > MPCR_MAX_EQ || m.nctrl > MPCR_MAX_CTRL ||
      m.nu > MPCR_MAX_ACT || m.nhullv > MPCR_MAX_HULLV || m.nhulla > MPCR_MAX_HULLA || m.nu < 0 || m.nhullv < 0 ||
      m.nhulla < 0)
    return fail(MPCR_EMODEL, "model exceeds blob capacity");
  if ((m.integrator != MPCR_INT_EULER && m.integrator != MPCR_INT_IMPLICITFAST) || (m.cone != MPCR_CONE_PYRAMIDAL && m.cone != MPCR_CONE_ELLIPTIC))
    return fail(MPCR_EMODEL, "only Euler / implicitfast with pyramidal or elliptic cones supported");
  if (m.nten < 0 || m.nten > MPCR_MAX_TEN) return fail(MPCR_EMODEL, "model exceeds blob capacity");
  if (m.density != 0) return fail(MPCR_EMODEL, "fluid density (inertia-box drag terms) not supported");
  if (m.viscosity != 0 && m.integrator != MPCR_INT_EULER)
    return fail(MPCR_EMODEL, "fluid viscosity with implicit integration not supported");
  for (int g = 0; g < m.ngeom; g++) {
    if (m.geom_hulladr[g] >= 0 && m.geom_hulladr[g] + m.geom_hullnum[g] > m.nhullv)
      return fail(MPCR_EMODEL, "geom %d hull outside the vertex table", g);
  }
  for (int v = 0; v < m.nhullv; v++)
    if (m.hull_adjadr[v] < 0 || m.hull_adjadr[v] + m.hull_adjnum[v] > m.nhulla)
      return fail(MPCR_EMODEL, "hull vertex %d adjacency outside the table", v);
  for (int k = 0; k < m.nhulla; k++)
    if (m.hull_adj[k] < 0 || m.hull_adj[k] >= m.nhullv) return fail(MPCR_EMODEL, "bad hull adjacency entry");
  for (int p = 0; p < m.npair; p++)
    for (int g : {m.pair_geom1[p], m.pair_geom2[p]})
      if (m.geom_type[g] == MPCR_GEOM_MESH && m.geom_hulladr[g] < 0)
        return fail(MPCR_EMODEL, "mesh geom %d in a pair has no convex hull", g);
  // polygon faces (v7): every index the manifold follows stays in its table
  if (m.nface < 0 || m.nface > MPCR_MAX_FACE || m.nfacev < 0 || m.nfacev > MPCR_MAX_FACEV || m.nvface < 0 ||
      m.nvface > MPCR_MAX_VFACE)
    return fail(MPCR_EMODEL, "model faces exceed blob capacity");
  for (int g = 0; g < m.ngeom; g++) {
    if (m.geom_faceadr[g] >= 0 && m.geom_faceadr[g] + m.geom_facenum[g] > m.nface)
      return fail(MPCR_EMODEL, "geom %d faces outside the face table", g);
    if (m.geom_cornadr[g] >= 0 && (m.geom_type[g] != MPCR_GEOM_BOX || m.geom_cornadr[g] + 8 > m.nhullv))
      return fail(MPCR_EMODEL, "geom %d box corners outside the vertex table", g);
    if (m.geom_faceadr[g] >= 0 && m.geom_type[g] == MPCR_GEOM_BOX && m.geom_cornadr[g] < 0)
      return fail(MPCR_EMODEL, "box geom %d has faces but no corners", g);
  }
  for (int f = 0; f < m.nface; f++)
    if (m.face_vadr[f] < 0 || m.face_vnum[f] < 3 || m.face_vnum[f] > MPCR_FACE_MAXV ||
        m.face_vadr[f] + m.face_vnum[f] > m.nfacev)
      return fail(MPCR_EMODEL, "face %d polygon outside the face-vertex table", f);
  for (int k = 0; k < m.nfacev; k++)
    if (m.face_vert[k] < 0 || m.face_vert[k] >= m.nhullv) return fail(MPCR_EMODEL, "bad face vertex entry");
  if (m.nface > 0)
    for (int v = 0; v < m.nhullv; v++)
      if (m.vert_faceadr[v] < 0 || m.vert_faceadr[v] + m.vert_facenum[v] > m.nvface)
        return fail(MPCR_EMODEL, "hull vertex %d face list outside the table", v);
  for (int k = 0; k < m.nvface; k++)
    if (m.vert_face[k] < 0 || m.vert_face[k] >= m.nface) return fail(MPCR_EMODEL, "bad vertex face entry");
  for (int p = 0; p < m.npair; p++)  // a polyhedron pair's geoms carry faces
    if (m.pair_func[p] == MPCR_COL_CONVEX && m.pair_ncon[p] == 4)
      for (int g : {m.pair_geom1[p], m.pair_geom2[p]})
        if (m.geom_faceadr[g] < 0) return fail(MPCR_EMODEL, "polyhedron-pair geom %d has no faces", g);
  return MPCR_OK;
}

extern "C" int mpcr_model_from_blob(const void* blob, size_t nbytes, mpcr_model** out) {
  if (!blob || !out) return fail(MPCR_EINVAL, "null argument");
  if (nbytes != sizeof(mpcr_model_t)) return fail(MPCR_EMODEL, "blob size %zu != %zu", nbytes, sizeof(mpcr_model_t));
  auto* h = new mpcr_model;
  std::memcpy(&h->m, blob, sizeof(mpcr_model_t));
  int rc = check_model(h->m);
  if (rc) { delete h; return rc; }
  *out = h;
  return MPCR_OK;
}

// MJCF: the compiler in libmpcr_mjcf.so (next to this library), dlopened on
// first use so the engine itself never links Python
static int load_mjcf(const char* path, double timestep, mpcr_model** out) {
  using compile_fn = int (*)(const char*, double, void**, size_t*, char*, int);
  using free_fn = void (*)(void*);
  static void* so = nullptr;
  if (!so) {
    Dl_info info;
    std::string dir = ".";
    if (dladdr(reinterpret_cast<void*>(&mpcr_model_load), &info) && info.dli_fname) {
      dir = info.dli_fname;
      size_t k = dir.find_last_of('/');
      dir = k == std::string::npos ? std::string(".") : dir.substr(0, k);
    }
    so = dlopen((dir + "/libmpcr_mjcf.so").c_str(), RTLD_NOW | RTLD_LOCAL);
    if (!so) return fail(MPCR_EMODEL, "MJCF compiler unavailable: %s", dlerror());
  }
  auto compile = reinterpret_cast<compile_fn>(dlsym(so, "mpcr_mjcf_compile"));
  auto release = reinterpret_cast<free_fn>(dlsym(so, "mpcr_mjcf_free"));
  if (!compile || !release) return fail(MPCR_EMODEL, "libmpcr_mjcf.so lacks its entry points");
  void* blob = nullptr;
  size_t n = 0;
  char err[512] = {0};
  if (compile(path, timestep, &blob, &n, err, sizeof(err)) != 0) return fail(MPCR_EMODEL, "MJCF %s: %s", path, err);
  int rc = mpcr_model_from_blob(blob, n, out);
  release(blob);
  return rc;
}

static bool is_mjcf(const char* path) {
  const size_t n = std::strlen(path);
  if (n >= 4 && std::strcmp(path + n - 4, ".xml") == 0) return true;
  FILE* f = fopen(path, "rb");
  if (!f) return false;
  int c;
  while ((c = fgetc(f)) == ' ' || c == '\n' || c == '\r' || c == '\t') {
  }
  fclose(f);
  return c == '<';
}

extern "C" int mpcr_model_load(const char* path, double timestep, mpcr_model** out) {
  if (!path || !out) return fail(MPCR_EINVAL, "null argument");
  if (is_mjcf(path)) return load_mjcf(path, timestep, out);
  FILE* f = fopen(path, "rb");
  if (!f) return fail(MPCR_EINVAL, "cannot open %s", path);
  std::vector<char> buf(sizeof(mpcr_model_t) + 1);
  size_t n = fread(buf.data(), 1, buf.size(), f);
  fclose(f);
  int rc = mpcr_model_from_blob(buf.data(), n, out);
  if (rc) return rc;
  if (timestep > 0) (*out)->m.timestep = timestep;
  return MPCR_OK;
}

extern "C" int mpcr_model_set_timestep(mpcr_model* m, double timestep) {
  if (!m || !(timestep > 0)) return fail(MPCR_EINVAL, "bad timestep");
  m->m.timestep = timestep;
  return MPCR_OK;
}

extern "C" int mpcr_model_info(const mpcr_model* m, int* nq, int* nv, int* nslot, int* nctrl, int* npair) {
  if (!m) return fail(MPCR_EINVAL, "null model");
  if (nq) *nq = m->m.nq;
  if (nv) *nv = m->m.nv;
  if (nslot) *nslot = m->m.nslot;
  if (nctrl) *nctrl = m->m.nctrl;
  if (npair) *npair = m->m.npair;
  return MPCR_OK;
}

extern "C" void mpcr_model_free(mpcr_model* m) { delete m; }

// ---- support start table (model v9: built here from hull_vert, not packed) ----
// Per hull and cube-map cell (6 faces x R x R, rollout.hip lut_cell order) the
// vertex extreme along the cell centre, in fp64.  The cells of a hull run in
// scan order, each climbing the hull graph (strict ascent) from the previous
// cell's vertex -- neighbouring cells mostly share one, so a cell costs a
// round or two -- and then taking the lowest index among the exactly tied
// maxima reachable along tied edges.  Any vertex of the hull would do as a
// start: the kernel's tie walk makes its supports start-independent
// (tests/test_gpu_parity.py), so R is a speed choice, and the extreme vertex
// keeps the climbs short and lets the engine mark cells exact.
static std::atomic<uint64_t> g_start_scramble{0};

static uint64_t mix64(uint64_t x) {  // splitmix64 finaliser
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

template <class F>
static void for_each_hull_parallel(const std::vector<int>& hulls, F&& f) {
  const int nt = (int)std::min<size_t>(hulls.size(), std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
  if (nt <= 1) {
    for (int g : hulls) f(g);
    return;
  }
  std::atomic<int> next{0};
  std::vector<std::thread> pool;
  for (int t = 0; t < nt; t++)
    pool.emplace_back([&] {
      for (int i; (i = next.fetch_add(1)) < (int)hulls.size();) f(hulls[i]);
    });
  for (auto& t : pool) t.join();
}

// geom_adr[ngeom]: each geom's first cell (-1: no hull); returns the cell
// count.  cells (nullable): the global vertex of every cell; scramble != 0
// names a hashed vertex of the hull instead (the start-independence tests).
static int64_t hull_start_table(const mpcr_model_t& m, int R, uint64_t scramble, int32_t* geom_adr,
                                int32_t* cells) {
  const int64_t nc = 6LL * R * R;
  int64_t n = 0;
  std::vector<int> hulls;
  std::vector<int64_t> first(m.ngeom, -1);
  for (int g = 0; g < m.ngeom; g++)
    if (m.geom_hulladr[g] >= 0 && m.geom_hullnum[g] > 0) {
      first[g] = n;
      n += nc;
      hulls.push_back(g);
    }
  if (geom_adr)
    for (int g = 0; g < m.ngeom; g++) geom_adr[g] = (int32_t)first[g];
  if (!cells) return n;
  std::vector<double> cen(R);
  for (int i = 0; i < R; i++) cen[i] = -1.0 + (2.0 * i + 1.0) / R;
  for_each_hull_parallel(hulls, [&](int g) {
    const int a = m.geom_hulladr[g], na = m.geom_hullnum[g];
    int32_t* out = cells + first[g];
    if (scramble) {
      for (int64_t c = 0; c < nc; c++) out[c] = a + (int)(mix64(scramble ^ ((uint64_t)g << 40) ^ (uint64_t)c) % na);
      return;
    }
    std::vector<int> tied;
    int v = a;
    for (int64_t c = 0; c < nc; c++) {
      const int f = (int)(c / ((int64_t)R * R)), iu = (int)((c / R) % R), iv = (int)(c % R), ax = f / 2;
      double d[3];
      d[ax] = (f & 1) ? -1.0 : 1.0;
      d[(ax + 1) % 3] = cen[iu];
      d[(ax + 2) % 3] = cen[iv];
      auto val = [&](int u) { return m.hull_vert[u][0] * d[0] + m.hull_vert[u][1] * d[1] + m.hull_vert[u][2] * d[2]; };
      double best = val(v);
      for (;;) {
        int nb = v;
        for (int k = m.hull_adjadr[v]; k < m.hull_adjadr[v] + m.hull_adjnum[v]; k++) {
          const int u = m.hull_adj[k];
          const double du = val(u);
          if (du > best) { best = du; nb = u; }
        }
        if (nb == v) break;
        v = nb;
      }
      tied.assign(1, v);
      int lo = v;
      for (size_t i = 0; i < tied.size() && tied.size() < 256; i++)
        for (int k = m.hull_adjadr[tied[i]]; k < m.hull_adjadr[tied[i]] + m.hull_adjnum[tied[i]]; k++) {
          const int u = m.hull_adj[k];
          if (val(u) == best && std::find(tied.begin(), tied.end(), u) == tied.end()) {
            tied.push_back(u);
            lo = std::min(lo, u);
          }
        }
      out[c] = lo;
    }
  });
  return n;
}

// exact[c] = 1 when cell c's start vertex is the support of every direction
// in the cell: the kernel's climb from it would end where it starts (no
// neighbour beats it, and no hint vertex beats the start), so the kernel skips
// the hint load and the climb -- bitwise the same support point, one
// dependent load instead of two or more.  A cube-map cell is the convex cone
// of its 4 corner rays and the directions a hull vertex is extreme for are a
// convex cone, bounded by its neighbours: the start vertex beats each
// neighbour by more than the margin along each corner ray (fp32 coordinates,
// as the kernel reads them), so along every direction of the cell.  The
// margin, max(1e-6 m, 32 FLT_EPSILON max|x|), scales with the hull's extent:
// the kernel's fp32 projections err by a few ulp of the largest coordinate
// (~1e-8 m on the gripper's cm-sized hulls, whose margin stays 1e-6 m;
// tests/test_hull_lut.py checks sampled directions on metre-sized hulls).
static void hull_exact_cells(const mpcr_model_t& m, int R, const int32_t* geom_adr, const int32_t* cells,
                             uint8_t* exact) {
  constexpr double kExactGap = 1e-6;
  std::vector<int> hulls;
  for (int g = 0; g < m.ngeom; g++)
    if (geom_adr[g] >= 0) hulls.push_back(g);
  auto xf = [&](int v, int k) { return (double)(float)m.hull_vert[v][k]; };
  for_each_hull_parallel(hulls, [&](int g) {
    double gap_min = kExactGap;
    for (int v = m.geom_hulladr[g]; v < m.geom_hulladr[g] + m.geom_hullnum[g]; v++)
      gap_min = std::max(gap_min, 32.0 * FLT_EPSILON * std::sqrt(xf(v, 0) * xf(v, 0) + xf(v, 1) * xf(v, 1) + xf(v, 2) * xf(v, 2)));
    for (int64_t c = 0, nc = 6LL * R * R; c < nc; c++) {
      const int v = cells[geom_adr[g] + c];
      const int f = (int)(c / ((int64_t)R * R)), iu = (int)((c / R) % R), iv = (int)(c % R), ax = f / 2;
      bool ok = true;
      for (int du = 0; du < 2 && ok; du++)
        for (int dv = 0; dv < 2 && ok; dv++) {
          double d[3];
          d[ax] = (f & 1) ? -1.0 : 1.0;
          d[(ax + 1) % 3] = -1.0 + 2.0 * (iu + du) / R;
          d[(ax + 2) % 3] = -1.0 + 2.0 * (iv + dv) / R;
          const double dn = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
          for (int k = m.hull_adjadr[v]; k < m.hull_adjadr[v] + m.hull_adjnum[v] && ok; k++) {
            const int u = m.hull_adj[k];
            const double gap = (xf(v, 0) - xf(u, 0)) * d[0] + (xf(v, 1) - xf(u, 1)) * d[1] + (xf(v, 2) - xf(u, 2)) * d[2];
            ok = gap > gap_min * dn;
          }
        }
      exact[geom_adr[g] + c] = ok;
    }
  });
}

extern "C" int64_t mpcr_model_hull_starts(const mpcr_model* m, int R, int32_t* geom_adr, int32_t* cells,
                                          uint8_t* exact, int64_t cap) {
  if (!m) return fail(MPCR_EINVAL, "null model");
  if (R == 0) R = MPCR_LUT_R;
  if (R < 1 || R > 1024) return fail(MPCR_EINVAL, "table resolution %d outside 1..1024", R);
  std::vector<int32_t> adr(std::max(1, m->m.ngeom));
  const int64_t n = hull_start_table(m->m, R, 0, adr.data(), nullptr);
  if (geom_adr) std::copy(adr.begin(), adr.begin() + m->m.ngeom, geom_adr);
  if ((cells || exact) && cap >= n) {
    std::vector<int32_t> own;
    if (!cells) own.resize(n), cells = own.data();
    hull_start_table(m->m, R, 0, nullptr, cells);
    if (exact) hull_exact_cells(m->m, R, adr.data(), cells, exact);
  }
  return n;
}

extern "C" uint64_t mpcr_set_hull_start_scramble(uint64_t seed) { return g_start_scramble.exchange(seed); }

// ---------------------------------------------------------------------------
// device model

static void h_qmul(double r[4], const double a[4], const double b[4]) {
  double t[4] = {a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
                 a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
                 a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
                 a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0]};
  std::memcpy(r, t, sizeof(t));
}
static void h_q2m(double m[9], const double q[4]) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  m[0] = 1 - 2 * (y * y + z * z); m[1] = 2 * (x * y - w * z); m[2] = 2 * (x * z + w * y);
  m[3] = 2 * (x * y + w * z); m[4] = 1 - 2 * (x * x + z * z); m[5] = 2 * (y * z - w * x);
  m[6] = 2 * (x * z - w * y); m[7] = 2 * (y * z + w * x); m[8] = 1 - 2 * (x * x + y * y);
}
static void h_rot(double r[3], const double q[4], const double v[3]) {
  double m[9];
  h_q2m(m, q);
  for (int i = 0; i < 3; i++) r[i] = m[3 * i] * v[0] + m[3 * i + 1] * v[1] + m[3 * i + 2] * v[2];
}

static int build_dev_model(const mpcr_model_t& m, const int32_t* lutadr, DevModel& d) {
  std::memset(&d, 0, sizeof(d));
  // dynamic bodies (not welded to the world), in topological order
  std::vector<int> dmap(m.nbody, -1);
  int nb = 0;
  for (int b = 1; b < m.nbody; b++)
    if (m.body_weldid[b] != 0) dmap[b] = nb++;
  if (nb > DX_NB) return fail(MPCR_EMODEL, "%d moving bodies > %d", nb, DX_NB);
  if (m.nv > DX_NV) return fail(MPCR_EMODEL, "nv=%d > %d (kernel solve width)", m.nv, DX_NV);
  if (m.nq > DX_NQ || m.njnt > DX_NJ || m.neq > DX_NEQ || m.nctrl > DX_NCTRL)
    return fail(MPCR_EMODEL, "model sizes exceed device capacity");
  // world poses of static bodies (constant)
  std::vector<double> wpos(3 * m.nbody, 0.0), wquat(4 * m.nbody, 0.0);
  wquat[0] = 1;
  for (int b = 1; b < m.nbody; b++) {
    if (m.body_weldid[b] != 0) continue;
    int p = m.body_parentid[b];
    double r[3];
    h_rot(r, &wquat[4 * p], m.body_pos[b]);
    for (int k = 0; k < 3; k++) wpos[3 * b + k] = wpos[3 * p + k] + r[k];
    h_qmul(&wquat[4 * b], &wquat[4 * p], m.body_quat[b]);
    double n = std::sqrt(wquat[4 * b] * wquat[4 * b] + wquat[4 * b + 1] * wquat[4 * b + 1] +
                         wquat[4 * b + 2] * wquat[4 * b + 2] + wquat[4 * b + 3] * wquat[4 * b + 3]);
    for (int k = 0; k < 4; k++) wquat[4 * b + k] /= n;
  }
  const bool no_passive = m.disableflags & MPCR_DSBL_PASSIVE;
  d.nbody = nb;
  d.njnt = m.njnt;
  d.nq = m.nq;
  d.nv = m.nv;
  d.neq = m.neq;
  d.nslot = m.nslot;
  d.nctrl = m.nctrl;
  d.iterations = m.iterations;
  d.ls_iterations = m.ls_iterations;
  d.disableflags = m.disableflags;
  d.timestep = (float)m.timestep;
  d.tolerance = (float)m.tolerance;
  d.ls_tolerance = (float)m.ls_tolerance;
  d.meaninertia = (float)m.meaninertia;
  const bool no_grav = m.disableflags & MPCR_DSBL_GRAVITY;
  for (int k = 0; k < 3; k++) d.gravity[k] = no_grav ? 0.f : (float)m.gravity[k];
  // trees
  std::vector<int> roots;
  std::vector<int> depth(m.nbody, 0);
  int maxdepth = 0;
  for (int b = 1; b < m.nbody; b++) {
    int i = dmap[b];
    if (i < 0) continue;
    int p = m.body_parentid[b];
    int njnt = m.body_jntnum[b];
    int j = njnt ? m.body_jntadr[b] : -1;
    if (njnt > 1) return fail(MPCR_EMODEL, "body %d has %d joints (1 supported)", b, njnt);
    if (j >= 0 && m.jnt_type[j] == MPCR_JNT_BALL) return fail(MPCR_EMODEL, "ball joints not supported");
    d.body_jnt[i] = j;
    d.body_kind[i] = j < 0 ? BK_WELD
                           : (m.jnt_type[j] == MPCR_JNT_FREE ? BK_FREE
                                                             : (m.jnt_type[j] == MPCR_JNT_HINGE ? BK_HINGE : BK_SLIDE));
    double bq[4], bp[3];
    if (dmap[p] < 0) {  // parent static: fold its constant world pose in
      double r[3];
      h_rot(r, &wquat[4 * p], m.body_pos[b]);
      for (int k = 0; k < 3; k++) bp[k] = wpos[3 * p + k] + r[k];
      h_qmul(bq, &wquat[4 * p], m.body_quat[b]);
      d.body_anc[i] = -1;
      depth[b] = 1;
    } else {
      std::memcpy(bp, m.body_pos[b], sizeof(bp));
      std::memcpy(bq, m.body_quat[b], sizeof(bq));
      d.body_anc[i] = dmap[p];
      depth[b] = depth[p] + 1;
    }
    if (d.body_kind[i] == BK_FREE) { d.body_anc[i] = -1; depth[b] = 1; }
    maxdepth = depth[b] > maxdepth ? depth[b] : maxdepth;
    for (int k = 0; k < 3; k++) d.body_bpos[i][k] = (float)bp[k];
    for (int k = 0; k < 4; k++) d.body_bquat[i][k] = (float)bq[k];
    for (int k = 0; k < 3; k++) d.body_ipos[i][k] = (float)m.body_ipos[b][k];
    double R[9];
    h_q2m(R, m.body_iquat[b]);
    double I[9];
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++)
        I[3 * r + c] = R[3 * r] * m.body_inertia[b][0] * R[3 * c] + R[3 * r + 1] * m.body_inertia[b][1] * R[3 * c + 1] +
                       R[3 * r + 2] * m.body_inertia[b][2] * R[3 * c + 2];
    d.body_Iloc[i][0] = (float)I[0]; d.body_Iloc[i][1] = (float)I[4]; d.body_Iloc[i][2] = (float)I[8];
    d.body_Iloc[i][3] = (float)I[1]; d.body_Iloc[i][4] = (float)I[2]; d.body_Iloc[i][5] = (float)I[5];
    d.body_mass[i] = (float)m.body_mass[b];
    d.body_gravcomp[i] = no_passive ? 0.f : (float)m.body_gravcomp[b];
    d.body_invw[i] = (float)m.body_invweight0[b][0];
    d.body_dofmask[i] = m.body_dofmask[b];
    int root = m.body_rootid[b];
    int t = -1;
    for (size_t k = 0; k < roots.size(); k++)
      if (roots[k] == root) t = (int)k;
    if (t < 0) { roots.push_back(root); t = (int)roots.size() - 1; }
    if (t >= DX_NTREE) return fail(MPCR_EMODEL, "too many kinematic trees");
    d.body_tree[i] = t;
    d.tree_mass[t] += (float)m.body_mass[b];
  }
  d.ntree = (int)roots.size();
  // inertia-box viscosity (mj_inertiaBoxFluidModel, density 0): the body's
  // equivalent box gives the diameter d = mean side
  if (m.viscosity > 0 && !no_passive)
    for (int b = 1; b < m.nbody; b++) {
      const int i = dmap[b];
      const double mass = m.body_mass[b];
      if (i < 0 || mass < 1e-15) continue;
      double diam = 0;
      for (int k = 0; k < 3; k++) {
        double x = m.body_inertia[b][(k + 1) % 3] + m.body_inertia[b][(k + 2) % 3] - m.body_inertia[b][k];
        diam += std::sqrt((x > 1e-15 ? x : 1e-15) / mass * 6) / 3;
      }
      d.body_visc[i][0] = (float)(-3 * M_PI * diam * m.viscosity);
      d.body_visc[i][1] = (float)(-M_PI * diam * diam * diam * m.viscosity);
    }
  // spatial tendons: site bodies and positions
  if (m.nten > DX_NTEN) return fail(MPCR_EMODEL, "%d spatial tendons > %d", m.nten, DX_NTEN);
  d.nten = m.nten;
  for (int t = 0; t < m.nten; t++) {
    for (int k = 0; k < 2; k++) {
      const int st = m.ten_site[t][k], b = m.site_bodyid[st];
      if (dmap[b] >= 0) {
        d.ten_body[t][k] = dmap[b];
        for (int c = 0; c < 3; c++) d.ten_pos[t][k][c] = (float)m.site_pos[st][c];
      } else {
        double r[3];
        h_rot(r, &wquat[4 * b], m.site_pos[st]);
        d.ten_body[t][k] = -1;
        for (int c = 0; c < 3; c++) d.ten_pos[t][k][c] = (float)(wpos[3 * b + c] + r[c]);
      }
    }
    d.ten_limited[t] = m.ten_limited[t];
    for (int k = 0; k < 2; k++) { d.ten_range[t][k] = (float)m.ten_range[t][k]; d.ten_solref[t][k] = (float)m.ten_solref[t][k]; }
    for (int k = 0; k < 5; k++) d.ten_solimp[t][k] = (float)m.ten_solimp[t][k];
    d.ten_margin[t] = (float)m.ten_margin[t];
    d.ten_invw[t] = (float)m.ten_invweight0[t];
  }
  d.cone = m.cone;
  d.impratio = (float)m.impratio;
  for (int t = 0; t < d.ntree; t++)
    if (d.tree_mass[t] <= 0) d.tree_mass[t] = 1.f;
  int rounds = 0;
  while ((1 << rounds) < maxdepth) rounds++;
  d.jump_rounds = rounds;
  // subtree masks (device body indices)
  for (int b = 1; b < m.nbody; b++) {
    if (dmap[b] < 0) continue;
    for (int a = b; a > 0; a = m.body_parentid[a])
      if (dmap[a] >= 0) d.body_submask[dmap[a]] |= 1u << dmap[b];
  }
  // joints
  for (int j = 0; j < m.njnt; j++) {
    d.jnt_type[j] = m.jnt_type[j];
    d.jnt_qposadr[j] = m.jnt_qposadr[j];
    d.jnt_dofadr[j] = m.jnt_dofadr[j];
    d.jnt_body[j] = dmap[m.jnt_bodyid[j]];
    d.jnt_limited[j] = m.jnt_limited[j];
    for (int k = 0; k < 3; k++) { d.jnt_pos[j][k] = (float)m.jnt_pos[j][k]; d.jnt_axis[j][k] = (float)m.jnt_axis[j][k]; }
    for (int k = 0; k < 2; k++) { d.jnt_range[j][k] = (float)m.jnt_range[j][k]; d.jnt_solref[j][k] = (float)m.jnt_solref[j][k]; }
    for (int k = 0; k < 5; k++) d.jnt_solimp[j][k] = (float)m.jnt_solimp[j][k];
    d.jnt_margin[j] = (float)m.jnt_margin[j];
    d.jnt_qpos0[j] = (float)m.qpos0[m.jnt_qposadr[j]];
  }
  // dofs
  for (int i = 0; i < m.nv; i++) {
    int j = m.dof_jntid[i];
    int b = m.dof_bodyid[i];
    d.dof_body[i] = dmap[b];
    d.dof_jnt[i] = j;
    int sub = i - m.jnt_dofadr[j];
    switch (m.jnt_type[j]) {
      case MPCR_JNT_HINGE: d.dof_kind[i] = 0; break;
      case MPCR_JNT_SLIDE: d.dof_kind[i] = 1; break;
      default: d.dof_kind[i] = sub < 3 ? 2 : 3; break;
    }
    d.dof_sub[i] = sub < 3 ? sub : sub - 3;
    uint32_t cm = 0;
    for (int a = i; a >= 0; a = m.dof_parentid[a]) cm |= 1u << a;
    d.dof_chainmask[i] = cm;
    int p = m.body_parentid[b];
    uint32_t pm = p > 0 ? m.body_dofmask[p] : 0u;
    if (m.jnt_type[j] == MPCR_JNT_FREE) {
      int d0 = m.jnt_dofadr[j];
      d.dof_velmask[i] = sub < 3 ? 0u : (pm | (7u << d0));
    } else {
      d.dof_velmask[i] = m.body_dofmask[b] & ~(1u << i);
    }
    d.dof_armature[i] = (float)m.dof_armature[i];
    d.dof_damping[i] = no_passive ? 0.f : (float)m.dof_damping[i];
    d.dof_invweight0[i] = (float)m.dof_invweight0[i];
  }
  for (int i = 0; i < m.nv; i++) d.dof_submask[i] = d.dof_body[i] >= 0 ? d.body_submask[d.dof_body[i]] : 0u;
  {  // blocked Cholesky layout: tree t's k-th dof (ascending) at lane 16 t + k
    int cnt[DX_NTREE] = {0}, mx = 0;
    bool ok = true;
    for (int l = 0; l < 64; l++) d.blane_dof[l] = -1;
    for (int i = 0; i < m.nv && ok; i++) {
      const int b = d.dof_body[i], t = b >= 0 ? d.body_tree[b] : -1;
      if (t < 0 || t >= DX_NTREE || cnt[t] >= 16) { ok = false; break; }
      d.blane_dof[16 * t + cnt[t]++] = i;
      mx = std::max(mx, cnt[t]);
    }
    d.blk_n = !ok ? 0 : (mx <= 8 ? 8 : 16);
    // rows spanning two trees keep Newton's H dense: equalities (joint: the
    // two joints' trees; connect: the two bodies', static = none) and tendons
    auto tree_of_body = [&](int b) { return b > 0 && dmap[b] >= 0 ? d.body_tree[dmap[b]] : -1; };
    auto cross = [](int t1, int t2) { return t1 >= 0 && t2 >= 0 && t1 != t2; };
    d.eq_cross = 0;
    for (int e = 0; e < m.neq; e++) {
      if (m.eq_type[e] == MPCR_EQ_JOINT) {
        const int j1 = m.eq_obj1[e], j2 = m.eq_obj2[e];
        if (j2 >= 0 && cross(tree_of_body(m.jnt_bodyid[j1]), tree_of_body(m.jnt_bodyid[j2]))) d.eq_cross = 1;
      } else if (m.eq_type[e] == MPCR_EQ_CONNECT) {
        if (cross(tree_of_body(m.eq_obj1[e]), tree_of_body(m.eq_obj2[e]))) d.eq_cross = 1;
      } else {
        d.eq_cross = 1;
      }
    }
    for (int t = 0; t < m.nten; t++)
      if (cross(tree_of_body(m.site_bodyid[m.ten_site[t][0]]), tree_of_body(m.site_bodyid[m.ten_site[t][1]])))
        d.eq_cross = 1;
  }
  {  // compact mass matrix (dual-arm image, SmemT::Mc): each tree's dofs contiguous
    int ts[DX_NTREE], te[DX_NTREE];
    bool ok = true;
    for (int t = 0; t < DX_NTREE; t++) ts[t] = te[t] = -1;
    for (int i = 0; i < m.nv && ok; i++) {
      const int b = d.dof_body[i], t = b >= 0 ? d.body_tree[b] : -1;
      if (t < 0 || t >= DX_NTREE) { ok = false; break; }
      if (ts[t] < 0) ts[t] = i;
      else if (te[t] != i) ok = false;  // a tree's dofs interleaved with another's
      te[t] = i + 1;
    }
    for (int i = 0; i < m.nv && ok; i++) {
      const int t = d.body_tree[d.dof_body[i]];
      d.mc_c0[i] = std::min(ts[t] & ~3, SmemW::NVW - SmemW::MCW);  // the window stays inside the NVW columns
      if (te[t] - d.mc_c0[i] > SmemW::MCW) ok = false;
    }
    d.mc_n = ok && m.nv * SmemW::MCW <= SmemW::MC ? m.nv : 0;
    if (env_int_or("MPCR_M_SLAB", 0)) d.mc_n = 0;  // tests: the HBM-slab path on a model that fits
    // the two-wave lead flush's pair limit; a lower one (tests) sends more steps to the dealt flush
    d.w2_lead_max = std::max(-1, std::min(W2_LEAD_MAX, env_int_or("MPCR_W2_LEAD_MAX", W2_LEAD_MAX)));
  }
  for (int i = 0; i < m.nq; i++) d.qpos_init[i] = (float)m.qpos_init[i];
  for (int i = 0; i < m.nv; i++) d.qvel_init[i] = (float)m.qvel_init[i];
  // collision geoms referenced by pairs
  std::vector<int> gmap(m.ngeom, -1);
  int ng = 0;
  for (int p = 0; p < m.npair; p++)
    for (int g : {m.pair_geom1[p], m.pair_geom2[p]})
      if (gmap[g] < 0) gmap[g] = ng++;
  if (ng > DX_NG || ng > WAVE) return fail(MPCR_EMODEL, "%d collision geoms > %d", ng, DX_NG < WAVE ? DX_NG : WAVE);
  d.ngeom = ng;
  for (int g = 0; g < m.ngeom; g++) {
    int i = gmap[g];
    if (i < 0) continue;
    int b = m.geom_bodyid[g];
    d.geom_type[i] = m.geom_type[g];
    d.geom_rbound[i] = (float)m.geom_rbound[g];
    d.geom_hulladr[i] = m.geom_hulladr[g];
    d.geom_hullnum[i] = m.geom_hullnum[g];
    d.geom_lutadr[i] = lutadr[g];
    d.geom_faceadr[i] = m.geom_faceadr[g];
    d.geom_facenum[i] = m.geom_faceadr[g] >= 0 ? m.geom_facenum[g] : 0;
    d.geom_cornadr[i] = m.geom_cornadr[g];
    for (int k = 0; k < 3; k++) d.geom_size[i][k] = (float)m.geom_size[g][k];
    if (dmap[b] >= 0) {
      d.geom_body[i] = dmap[b];
      for (int k = 0; k < 3; k++) d.geom_pos[i][k] = (float)m.geom_pos[g][k];
      for (int k = 0; k < 4; k++) d.geom_quat[i][k] = (float)m.geom_quat[g][k];
    } else {  // static geom: store its world pose
      d.geom_body[i] = -1;
      double r[3], q[4];
      h_rot(r, &wquat[4 * b], m.geom_pos[g]);
      h_qmul(q, &wquat[4 * b], m.geom_quat[g]);
      for (int k = 0; k < 3; k++) d.geom_pos[i][k] = (float)(wpos[3 * b + k] + r[k]);
      for (int k = 0; k < 4; k++) d.geom_quat[i][k] = (float)q[k];
    }
  }
  // pairs
  if (m.npair > DX_NP) return fail(MPCR_EMODEL, "too many pairs");
  if (m.nslot > DX_NSLOT) return fail(MPCR_EMODEL, "%d masked slots > %d", m.nslot, DX_NSLOT);
  d.npair = m.npair;
  d.cvx_base = m.npair;
  for (int p = m.npair - 1; p >= 0; p--)
    if (m.pair_func[p] >= MPCR_COL_CONVEX) d.cvx_base = p;
  for (int p = d.cvx_base; p < m.npair; p++)
    if (m.pair_func[p] < MPCR_COL_CONVEX) return fail(MPCR_EMODEL, "convex pairs must be sorted last");
  if (m.npair - d.cvx_base > 512) return fail(MPCR_EMODEL, "%d general-convex pairs > 512", m.npair - d.cvx_base);
  d.coll_rows = m.npair <= WAVE;  // DevModel::coll_rows: a light collision phase
  for (int p = 0; p < m.npair; p++)
    if (m.pair_func[p] == MPCR_COL_BOX_BOX) d.coll_rows = 0;
  d.cvx_joint = 1;  // DevModel::cvx_joint: no convex pair carries a cost slot
  for (int p = d.cvx_base; p < m.npair; p++)
    if (m.pair_slotadr[p] >= 0) d.cvx_joint = 0;
  if (m.nhullv > 32767) return fail(MPCR_EMODEL, "hull vertex table exceeds 16-bit hints");
  for (int p = 0; p < m.npair; p++) {
    int g1 = m.pair_geom1[p], g2 = m.pair_geom2[p];
    d.pair_g1[p] = gmap[g1];
    d.pair_g2[p] = gmap[g2];
    d.pair_func[p] = m.pair_func[p];
    if (m.pair_func[p] == MPCR_COL_BOX_BOX && m.pair_slotadr[p] >= 0)
      return fail(MPCR_EMODEL, "robot-masked box-box pairs are not supported by the kernel");
    d.pair_ncon[p] = m.pair_ncon[p];
    d.pair_slotadr[p] = m.pair_slotadr[p];
    d.pair_condim[p] = m.pair_condim[p];
    d.pair_friction[p] = (float)m.pair_friction[p];
    d.pair_cmu[p] = (float)(m.pair_friction[p] / std::sqrt(m.impratio > 0 ? m.impratio : 1.0));
    if (m.pair_condim[p] != 1 && m.pair_condim[p] != 3) return fail(MPCR_EMODEL, "condim %d not supported", m.pair_condim[p]);
    d.pair_margin[p] = (float)(m.pair_margin[p] - m.pair_gap[p]);
    for (int k = 0; k < 2; k++) d.pair_solref[p][k] = (float)m.pair_solref[p][k];
    for (int k = 0; k < 5; k++) d.pair_solimp[p][k] = (float)m.pair_solimp[p][k];
    d.pair_diag[p] = (float)(m.body_invweight0[m.geom_bodyid[g1]][0] + m.body_invweight0[m.geom_bodyid[g2]][0]);
    const int b1 = d.geom_body[d.pair_g1[p]], b2 = d.geom_body[d.pair_g2[p]];
    d.pair_jinfo[p] = make_int4(b1 >= 0 ? (int)d.body_dofmask[b1] : 0, b2 >= 0 ? (int)d.body_dofmask[b2] : 0,
                                b1 >= 0 ? d.body_tree[b1] : 0, b2 >= 0 ? d.body_tree[b2] : 0);
  }
  // equalities: joint (1 row) and connect (3 rows), rows in model order
  int nrow = 0;
  for (int e = 0; e < m.neq; e++) {
    d.eq_type[e] = m.eq_type[e];
    for (int k = 0; k < 5; k++) d.eq_solimp[e][k] = (float)m.eq_solimp[e][k];
    for (int k = 0; k < 2; k++) d.eq_solref[e][k] = (float)m.eq_solref[e][k];
    if (m.eq_type[e] == MPCR_EQ_JOINT) {
      d.eq_j1[e] = m.eq_obj1[e];
      d.eq_j2[e] = m.eq_obj2[e];
      for (int k = 0; k < 5; k++) d.eq_data[e][k] = (float)m.eq_data[e][k];
      double diag = m.dof_invweight0[m.jnt_dofadr[m.eq_obj1[e]]];
      if (m.eq_obj2[e] >= 0) diag += m.dof_invweight0[m.jnt_dofadr[m.eq_obj2[e]]];
      d.eq_diag[e] = (float)diag;
      if (nrow + 1 > DX_NEQROW) return fail(MPCR_EMODEL, "too many equality rows");
      d.eqrow_eq[nrow] = e; d.eqrow_k[nrow] = 0; nrow++;
    } else if (m.eq_type[e] == MPCR_EQ_CONNECT) {
      for (int side = 0; side < 2; side++) {
        int b = side ? m.eq_obj2[e] : m.eq_obj1[e];
        const double* a = m.eq_data[e] + 3 * side;
        int db = b > 0 ? dmap[b] : -1;
        (side ? d.eq_b2 : d.eq_b1)[e] = db;
        double pw[3] = {a[0], a[1], a[2]};
        if (db < 0) {  // static body: anchor in world once
          double r[3];
          h_rot(r, &wquat[4 * b], a);
          for (int k = 0; k < 3; k++) pw[k] = wpos[3 * b + k] + r[k];
        }
        for (int k = 0; k < 3; k++) d.eq_data[e][4 * side + k] = (float)pw[k];
      }
      d.eq_diag[e] = (float)(m.body_invweight0[m.eq_obj1[e]][0] + m.body_invweight0[m.eq_obj2[e]][0]);
      if (nrow + 3 > DX_NEQROW) return fail(MPCR_EMODEL, "too many equality rows");
      for (int k = 0; k < 3; k++) { d.eqrow_eq[nrow] = e; d.eqrow_k[nrow] = k + 1; nrow++; }
    } else {
      return fail(MPCR_EMODEL, "equality type %d not supported (joint, connect)", m.eq_type[e]);
    }
  }
  d.neqrow = nrow;
  // springs
  for (int i = 0; i < m.nv; i++) {
    int j = m.dof_jntid[i];
    d.dof_qposadr[i] = m.jnt_qposadr[j];
    if (!no_passive && (m.jnt_type[j] == MPCR_JNT_HINGE || m.jnt_type[j] == MPCR_JNT_SLIDE) &&
        m.jnt_stiffness[j] != 0) {
      d.dof_stiffness[i] = (float)m.jnt_stiffness[j];
      d.dof_springref[i] = (float)m.jnt_springref[j];
      d.has_spring = 1;
    }
    d.dof_actfrc[i][0] = -3e38f;
    d.dof_actfrc[i][1] = 3e38f;
    if (m.jnt_actfrclimited[j]) {
      d.dof_actfrc[i][0] = (float)m.jnt_actfrcrange[j][0];
      d.dof_actfrc[i][1] = (float)m.jnt_actfrcrange[j][1];
    }
  }
  // actuators (ctrl constant: clamped once here)
  if (m.nu > DX_NU) return fail(MPCR_EMODEL, "%d actuators > %d", m.nu, DX_NU);
  d.nu = m.nu;
  for (int a = 0; a < m.nu; a++) {
    d.act_ntrn[a] = m.act_ntrn[a];
    for (int k = 0; k < m.act_ntrn[a]; k++) {
      int v = m.act_dof[a][k];
      d.act_dof[a][k] = v;
      d.act_qadr[a][k] = m.act_qadr[a][k];
      d.act_moment[a][k] = (float)m.act_moment[a][k];
      if (d.dof_actn[v] >= 2) return fail(MPCR_EMODEL, "more than 2 actuators on dof %d", v);
      d.dof_acta[v][d.dof_actn[v]] = a;
      d.dof_actm[v][d.dof_actn[v]] = (float)m.act_moment[a][k];
      d.dof_actn[v]++;
    }
    double ctrl = m.act_ctrl[a];
    if (m.act_ctrllimited[a]) ctrl = std::fmin(std::fmax(ctrl, m.act_ctrlrange[a][0]), m.act_ctrlrange[a][1]);
    d.act_gaffine[a] = m.act_gaintype[a] == MPCR_GAIN_AFFINE;
    d.act_baffine[a] = m.act_biastype[a] == MPCR_BIAS_AFFINE;
    for (int k = 0; k < 3; k++) { d.act_gain[a][k] = (float)m.act_gainprm[a][k]; d.act_bias[a][k] = (float)m.act_biasprm[a][k]; }
    d.act_gain[a][3] = (float)ctrl;
    d.act_frc[a][0] = m.act_forcelimited[a] ? (float)m.act_forcerange[a][0] : -3e38f;
    d.act_frc[a][1] = m.act_forcelimited[a] ? (float)m.act_forcerange[a][1] : 3e38f;
  }
  // implicitfast: D = -qDeriv = damping + sum_a (-dforce/dvel) m m^T (fp64, then rounded)
  d.integrator = m.integrator;
  if (m.integrator == MPCR_INT_IMPLICITFAST) {
    std::vector<double> D((size_t)m.nv * m.nv, 0.0);
    for (int i = 0; i < m.nv; i++) D[(size_t)i * m.nv + i] = no_passive ? 0.0 : m.dof_damping[i];
    for (int a = 0; a < m.nu; a++) {
      double dv = 0;
      if (m.act_biastype[a] == MPCR_BIAS_AFFINE) dv += m.act_biasprm[a][2];
      if (m.act_gaintype[a] == MPCR_GAIN_AFFINE) dv += m.act_gainprm[a][2] * (double)d.act_gain[a][3];
      for (int k = 0; k < m.act_ntrn[a]; k++)
        for (int l = 0; l < m.act_ntrn[a]; l++)
          D[(size_t)m.act_dof[a][k] * m.nv + m.act_dof[a][l]] -= dv * m.act_moment[a][k] * m.act_moment[a][l];
    }
    for (int i = 0; i < m.nv; i++)
      for (int j = 0; j < m.nv; j++) d.impl_D[i][j] = (float)D[(size_t)i * m.nv + j];
    d.impl_cross = 0;  // a transmission across trees keeps the implicit solve dense
    for (int i = 0; i < m.nv; i++)
      for (int j = 0; j < m.nv; j++)
        if (D[(size_t)i * m.nv + j] != 0.0 && d.body_tree[d.dof_body[i]] != d.body_tree[d.dof_body[j]]) d.impl_cross = 1;
  } else if (m.integrator != MPCR_INT_EULER) {
    return fail(MPCR_EMODEL, "integrator %d not supported (Euler, implicitfast)", m.integrator);
  }
  // planner ids
  d.hande_body = m.hande_body >= 0 ? dmap[m.hande_body] : -1;
  d.tcp_body = -1;
  if (m.tcp_site >= 0) {
    d.tcp_body = dmap[m.site_bodyid[m.tcp_site]];
    for (int k = 0; k < 3; k++) d.tcp_pos[k] = (float)m.site_pos[m.tcp_site][k];
  }
  for (int k = 0; k < m.nctrl; k++) { d.ctrl_qposadr[k] = m.ctrl_qposadr[k]; d.ctrl_dofadr[k] = m.ctrl_dofadr[k]; }
  return MPCR_OK;
}

// ---------------------------------------------------------------------------
// engines

extern "C" int mpcr_engine_create(const mpcr_model* m, int device, int max_n, int horizon, const float* pdot,
                                  int nbasis, mpcr_engine** out) {
  if (!m || !out || max_n <= 0 || horizon <= 0 || !pdot || nbasis <= 0 || nbasis > 12)
    return fail(MPCR_EINVAL, "bad engine arguments");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(MPCR_ENODEV, "no HIP device");
  if (device < 0 || device >= ndev) return fail(MPCR_ENODEV, "device %d out of range (%d)", device, ndev);
  HIPCHK(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(MPCR_ENODEV, "device %d is %s; libmpcr is built for gfx950 only", device, prop.gcnArchName);
  auto* e = new mpcr_engine;
  e->device = device;
  e->max_n = max_n;
  e->H = horizon;
  e->nbasis = nbasis;
  e->host = m->m;
  std::vector<int32_t> lutadr(std::max(1, e->host.ngeom));
  const int64_t nlut = hull_start_table(e->host, MPCR_LUT_R, 0, lutadr.data(), nullptr);
  int rc = build_dev_model(e->host, lutadr.data(), e->dev);
  if (rc) { delete e; return rc; }
  e->wide = needs_wide(e->host, e->dev);
  if (e->host.nhullv > 0) {  // hull vertices (float4) + graph, pointed to by the device model
    const mpcr_model_t& h = e->host;
    std::vector<float4> hv(h.nhullv);
    std::vector<int2> hi(h.nhullv);
    std::vector<float4> ha(h.nhulla);
    std::vector<float4> hh((size_t)h.nhullv * 8);
    if (h.nhullv > 65535) {
      mpcr_engine_free(e);
      return fail(MPCR_EINVAL, "%d hull vertices: the climb records hold 16-bit vertex indices", h.nhullv);
    }
    auto bitsf = [](int bits) {
      float f;
      std::memcpy(&f, &bits, 4);
      return f;
    };
    // neighbour record: xyz | index | degree << 16 -- the chosen neighbour's
    // own adjacency is then addressed without another dependent load
    auto rec = [&](int u) {
      return make_float4((float)h.hull_vert[u][0], (float)h.hull_vert[u][1], (float)h.hull_vert[u][2],
                         bitsf(u | (h.hull_adjnum[u] << 16)));
    };
    for (int k = 0; k < h.nhulla; k++) ha[k] = rec(h.hull_adj[k]);
    const float nan = std::numeric_limits<float>::quiet_NaN();
    for (int v = 0; v < h.nhullv; v++) {
      hv[v] = make_float4((float)h.hull_vert[v][0], (float)h.hull_vert[v][1], (float)h.hull_vert[v][2],
                          bitsf(h.hull_adjnum[v]));
      hi[v] = make_int2(h.hull_adjadr[v], h.hull_adjnum[v]);
      for (int j = 0; j < 8; j++)  // NaN pads never beat the current vertex
        hh[(size_t)v * 8 + j] = j < h.hull_adjnum[v] ? rec(h.hull_adj[h.hull_adjadr[v] + j]) : make_float4(nan, nan, nan, bitsf(-1));
    }
    if (hipMalloc(&e->d_hull_vert, sizeof(float4) * hv.size()) != hipSuccess ||
        hipMalloc(&e->d_hull_info, sizeof(int2) * hi.size()) != hipSuccess ||
        hipMalloc(&e->d_hull_adjv, sizeof(float4) * (ha.size() ? ha.size() : 1)) != hipSuccess ||
        hipMalloc(&e->d_hull_head, sizeof(float4) * hh.size()) != hipSuccess ||
        hipMemcpy(e->d_hull_vert, hv.data(), sizeof(float4) * hv.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(e->d_hull_info, hi.data(), sizeof(int2) * hi.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(e->d_hull_head, hh.data(), sizeof(float4) * hh.size(), hipMemcpyHostToDevice) != hipSuccess ||
        (ha.size() && hipMemcpy(e->d_hull_adjv, ha.data(), sizeof(float4) * ha.size(), hipMemcpyHostToDevice) != hipSuccess)) {
      mpcr_engine_free(e);
      return fail(MPCR_ENOMEM, "hull upload failed");
    }
    e->dev.hull_vert = as_gmem(e->d_hull_vert);
    e->dev.hull_info = as_gmem(e->d_hull_info);
    e->dev.hull_adjv = as_gmem(e->d_hull_adjv);
    e->dev.hull_head = as_gmem(e->d_hull_head);
    // the support start table, exact cells flagged in bit 15 of the record's
    // index half (vertex indices are < 32768; hull_exact_cells)
    std::vector<int32_t> cells(nlut);
    std::vector<uint8_t> exact(nlut);
    hull_start_table(h, MPCR_LUT_R, g_start_scramble.load(), nullptr, cells.data());
    hull_exact_cells(h, MPCR_LUT_R, lutadr.data(), cells.data(), exact.data());
    std::vector<float4> hl(nlut > 0 ? nlut : 1);
    for (int64_t c = 0; c < nlut; c++) {
      const int v = cells[c];
      hl[c] = rec(v);
      if (exact[c]) hl[c].w = bitsf(v | 0x8000 | (h.hull_adjnum[v] << 16));
    }
    if (hipMalloc(&e->d_hull_lut, sizeof(float4) * (nlut ? nlut : 1)) != hipSuccess ||
        (nlut && hipMemcpy(e->d_hull_lut, hl.data(), sizeof(float4) * nlut, hipMemcpyHostToDevice) != hipSuccess)) {
      mpcr_engine_free(e);
      return fail(MPCR_ENOMEM, "hull table upload failed");
    }
    e->dev.hull_lut = as_gmem(e->d_hull_lut);
  }
  if (e->host.nface > 0) {  // polygon faces + vertex incidence, pointed to by the device model
    const mpcr_model_t& h = e->host;
    std::vector<float4> fp(h.nface);
    std::vector<int2> fv(h.nface), vf(h.nhullv);
    for (int f = 0; f < h.nface; f++) {
      fp[f] = make_float4((float)h.face_plane[f][0], (float)h.face_plane[f][1], (float)h.face_plane[f][2],
                          (float)h.face_plane[f][3]);
      fv[f] = make_int2(h.face_vadr[f], h.face_vnum[f]);
    }
    for (int v = 0; v < h.nhullv; v++) vf[v] = make_int2(h.vert_faceadr[v], h.vert_facenum[v]);
    if (hipMalloc(&e->d_face_plane, sizeof(float4) * fp.size()) != hipSuccess ||
        hipMalloc(&e->d_face_vinfo, sizeof(int2) * fv.size()) != hipSuccess ||
        hipMalloc(&e->d_face_vert, sizeof(int) * h.nfacev) != hipSuccess ||
        hipMalloc(&e->d_vert_finfo, sizeof(int2) * vf.size()) != hipSuccess ||
        hipMalloc(&e->d_vert_face, sizeof(int) * h.nvface) != hipSuccess ||
        hipMemcpy(e->d_face_plane, fp.data(), sizeof(float4) * fp.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(e->d_face_vinfo, fv.data(), sizeof(int2) * fv.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(e->d_face_vert, h.face_vert, sizeof(int) * h.nfacev, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(e->d_vert_finfo, vf.data(), sizeof(int2) * vf.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(e->d_vert_face, h.vert_face, sizeof(int) * h.nvface, hipMemcpyHostToDevice) != hipSuccess) {
      mpcr_engine_free(e);
      return fail(MPCR_ENOMEM, "face upload failed");
    }
    e->dev.face_plane = as_gmem(e->d_face_plane);
    e->dev.face_vinfo = as_gmem(e->d_face_vinfo);
    e->dev.face_vert = as_gmem(e->d_face_vert);
    e->dev.vert_finfo = as_gmem(e->d_vert_finfo);
    e->dev.vert_face = as_gmem(e->d_vert_face);
    // the polyhedron manifold's cone table: per geom with faces and per
    // cube-map cell of the local direction (CONE_R x CONE_R per cube face, the
    // kernel's cone_cell order) every face whose outward normal lies within
    // acos(CONE_COS) + the cell's angular radius + 0.01 rad of the cell centre
    // -- a superset of the faces the kernel's cone test accepts for any
    // direction in the cell (fp32 cell assignment included), ascending, so the
    // scan of a cell's list compacts the same candidates in the same order as a
    // scan of all the geom's faces
    std::vector<int2> ccell;
    std::vector<int> cface;
    const double thr0 = std::acos(CONE_COS) + 0.01;
    for (int i = 0; i < e->dev.ngeom; i++) {
      e->dev.geom_coneadr[i] = -1;
      const int fa = e->dev.geom_faceadr[i], fnum = e->dev.geom_facenum[i];
      if (fa < 0 || fnum <= 0) continue;
      e->dev.geom_coneadr[i] = (int)ccell.size();
      for (int c = 0; c < CONE_CELLS; c++) {
        const int fc = c / (CONE_R * CONE_R), iu = (c / CONE_R) % CONE_R, iv = c % CONE_R;
        const int ax = fc / 2;
        const double sa = (fc & 1) ? -1.0 : 1.0;
        auto dir = [&](double u, double v, double out[3]) {
          out[ax] = sa; out[(ax + 1) % 3] = u; out[(ax + 2) % 3] = v;
          const double nn = std::sqrt(out[0] * out[0] + out[1] * out[1] + out[2] * out[2]);
          for (int k = 0; k < 3; k++) out[k] /= nn;
        };
        const double u0 = -1.0 + 2.0 * iu / CONE_R, u1 = -1.0 + 2.0 * (iu + 1) / CONE_R;
        const double v0 = -1.0 + 2.0 * iv / CONE_R, v1 = -1.0 + 2.0 * (iv + 1) / CONE_R;
        double ctr[3], cr[3];
        dir(0.5 * (u0 + u1), 0.5 * (v0 + v1), ctr);
        double rad = 0.0;
        for (double u : {u0, u1})
          for (double v : {v0, v1}) {
            dir(u, v, cr);
            const double cd = ctr[0] * cr[0] + ctr[1] * cr[1] + ctr[2] * cr[2];
            rad = std::max(rad, std::acos(std::min(1.0, cd)));
          }
        const double cth = std::cos(thr0 + rad);
        const int start = (int)cface.size();
        for (int f = fa; f < fa + fnum; f++) {
          const double* fp = h.face_plane[f];
          const double fn = std::sqrt(fp[0] * fp[0] + fp[1] * fp[1] + fp[2] * fp[2]);
          if (fn > 0 && (fp[0] * ctr[0] + fp[1] * ctr[1] + fp[2] * ctr[2]) / fn >= cth) cface.push_back(f);
        }
        ccell.push_back(make_int2(start, (int)cface.size() - start));
      }
    }
    if (cface.empty()) cface.push_back(0);
    if (ccell.empty()) ccell.push_back(make_int2(0, 0));
    if (hipMalloc(&e->d_cone_cell, sizeof(int2) * ccell.size()) != hipSuccess ||
        hipMalloc(&e->d_cone_face, sizeof(int) * cface.size()) != hipSuccess ||
        hipMemcpy(e->d_cone_cell, ccell.data(), sizeof(int2) * ccell.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(e->d_cone_face, cface.data(), sizeof(int) * cface.size(), hipMemcpyHostToDevice) != hipSuccess) {
      mpcr_engine_free(e);
      return fail(MPCR_ENOMEM, "cone table upload failed");
    }
    e->dev.cone_cell = as_gmem(e->d_cone_cell);
    e->dev.cone_face = as_gmem(e->d_cone_face);
  }
  const int nc = e->host.nctrl;
  const size_t in_cols = (size_t)nc * (horizon > nbasis ? horizon : nbasis);
  if (hipMalloc(&e->d_model, sizeof(DevModel)) != hipSuccess ||
      hipMalloc(&e->d_pdot, sizeof(float) * horizon * nbasis) != hipSuccess ||
      hipMalloc(&e->d_in, sizeof(float) * max_n * in_cols) != hipSuccess ||
      hipMalloc(&e->d_cost, sizeof(float) * max_n * 4) != hipSuccess ||
      hipMalloc(&e->d_theta, sizeof(float) * max_n * nc * horizon) != hipSuccess ||
      hipMalloc(&e->d_thetadot, sizeof(float) * max_n * nc * horizon) != hipSuccess ||
      hipMalloc(&e->d_key, sizeof(unsigned long long)) != hipSuccess ||
      hipMalloc(&e->d_status, sizeof(int) * max_n) != hipSuccess ||
      hipMalloc(&e->d_idx, sizeof(int) * max_n) != hipSuccess ||
      // per-candidate scratch slabs: one spare row for the empty group of a
      // two-candidate wave (narrow kernel, odd n)
      hipMalloc(&e->d_slot_prev, sizeof(float) * ((size_t)max_n + 1) * (e->host.nslot > 0 ? e->host.nslot : 1)) !=
          hipSuccess ||
      hipMalloc(&e->d_jx, sizeof(float) * ((size_t)max_n + 1) *
                              (e->wide ? (SmemW::MAXEFC - SmemW::JL + 1) * SmemW::LDJ
                                       : (SmemN::MAXEFC - SmemN::JL + 1) * SmemN::LDJ)) !=
          hipSuccess ||
      hipMalloc(&e->d_hints, sizeof(short) * 2 * (size_t)max_n * (e->wide ? SmemW::NHINT : 1)) != hipSuccess ||
      hipMalloc(&e->d_pace, sizeof(unsigned) * MPCR_PACE_SLOTS) != hipSuccess ||
      hipMalloc(&e->d_mslab, sizeof(float) * ((size_t)max_n + 1) * (e->wide ? SmemW::NVW * SmemW::LD : 1)) !=
          hipSuccess ||
      hipMalloc(&e->d_td, sizeof(float) * ((size_t)max_n + 1) * (size_t)(e->host.nctrl > 0 ? e->host.nctrl : 1) *
                              (size_t)horizon) != hipSuccess) {
    mpcr_engine_free(e);
    return fail(MPCR_ENOMEM, "device allocation failed");
  }
  if (hipMemcpy(e->d_model, &e->dev, sizeof(DevModel), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(e->d_pdot, pdot, sizeof(float) * horizon * nbasis, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(e->d_hints, 0xff, sizeof(short) * 2 * (size_t)max_n * (e->wide ? SmemW::NHINT : 1)) !=
          hipSuccess ||
      hipMemset(e->d_pace, 0xff, sizeof(unsigned) * MPCR_PACE_SLOTS) != hipSuccess) {
    mpcr_engine_free(e);
    return fail(MPCR_EHIP, "model upload failed");
  }
  if (e->wide) {
    // horizon segments (MPCR_SEG_STEPS / MPCR_SEG_GROUPS override the defaults)
    e->seg_steps = env_int_or("MPCR_SEG_STEPS", MPCR_SEG_STEPS_DEFAULT);
    e->seg_groups = std::max(1, std::min(MPCR_SEG_MAXG, env_int_or("MPCR_SEG_GROUPS", MPCR_SEG_GROUPS_DEFAULT)));
    if (e->seg_steps > 0 && e->seg_steps < horizon) {
      // a batch the device holds in one round gains nothing: its blocks all
      // start together (the one-wave variant's resident blocks per CU x CUs)
      int occ[6] = {0, 0, 0, 0, 0, 0}, ncu = 0;
      if (rollout_occupancy(occ, MPCR_N_DYN_LDS) == hipSuccess &&
          hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess)
        e->seg_min_n = occ[3] * ncu;
      bool ok = hipMalloc(&e->d_seg, sizeof(float) * (size_t)max_n * SEG_STRIDE) == hipSuccess;
      for (int g = 0; ok && e->seg_groups > 1 && g < e->seg_groups; g++)
        ok = hipStreamCreateWithFlags(&e->seg_stream[g], hipStreamNonBlocking) == hipSuccess;
      for (int g = 0; ok && e->seg_groups > 1 && g <= e->seg_groups; g++)
        ok = hipEventCreateWithFlags(&e->seg_event[g], hipEventDisableTiming) == hipSuccess;
      if (!ok) {
        mpcr_engine_free(e);
        return fail(MPCR_ENOMEM, "horizon-segment state allocation failed");
      }
    }
  }
  *out = e;
  return MPCR_OK;
}

extern "C" void mpcr_engine_free(mpcr_engine* e) {
  if (!e) return;
  (void)hipFree(e->d_model);
  (void)hipFree(e->d_pdot);
  (void)hipFree(e->d_in);
  (void)hipFree(e->d_cost);
  (void)hipFree(e->d_theta);
  (void)hipFree(e->d_thetadot);
  (void)hipFree(e->d_key);
  (void)hipFree(e->d_status);
  (void)hipFree(e->d_idx);
  (void)hipFree(e->d_slot_prev);
  (void)hipFree(e->d_jx);
  (void)hipFree(e->d_td);
  (void)hipFree(e->d_hints);
  (void)hipFree(e->d_pace);
  (void)hipFree(e->d_mslab);
  (void)hipFree(e->d_seg);
  for (int g = 0; g < MPCR_SEG_MAXG; g++)
    if (e->seg_stream[g]) (void)hipStreamDestroy(e->seg_stream[g]);
  for (int g = 0; g <= MPCR_SEG_MAXG; g++)
    if (e->seg_event[g]) (void)hipEventDestroy(e->seg_event[g]);
  (void)hipFree(e->d_face_plane);
  (void)hipFree(e->d_face_vinfo);
  (void)hipFree(e->d_face_vert);
  (void)hipFree(e->d_vert_finfo);
  (void)hipFree(e->d_vert_face);
  (void)hipFree(e->d_cone_cell);
  (void)hipFree(e->d_cone_face);
  (void)hipFree(e->d_hull_vert);
  (void)hipFree(e->d_hull_info);
  (void)hipFree(e->d_hull_adjv);
  (void)hipFree(e->d_hull_head);
  (void)hipFree(e->d_hull_lut);
  delete e;
}

// per-call parameter block of the kernel (RolloutArgs::par layout)
static void fill_par(float* par, int nc, const double* q0, const float* w, const float* ptgt, const float* qtgt) {
  for (int k = 0; k < PAR_N; k++) par[k] = 0.f;
  if (q0)
    for (int k = 0; k < nc; k++) par[PAR_Q0 + k] = (float)q0[k];
  for (int k = 0; k < 3; k++) { par[PAR_W + k] = w[k]; par[PAR_PT + k] = ptgt[k]; }
  for (int k = 0; k < 4; k++) par[PAR_QT + k] = qtgt[k];
}

struct Launch {
  const float* in = nullptr;
  int layout = 0, n = 0, index_base = 0, plant = 0;
  const float* dpar = nullptr;  // device parameter block (else par)
  float par[PAR_N] = {};
  float* state = nullptr;
  float *cost4 = nullptr, *theta = nullptr, *thetadot = nullptr, *trace_eef = nullptr, *trace_slots = nullptr;
  unsigned long long* key = nullptr;
  int* status = nullptr;
  float* dbg = nullptr;
  bool reset_key = false;
};

static int launch_rollout(mpcr_engine* e, const Launch& l, hipStream_t st) {
  RolloutArgs a;
  std::memset(&a, 0, sizeof(a));
  a.m = e->d_model;
  a.input = l.in;
  a.pdot = e->d_pdot;
  a.cost4 = l.cost4;
  a.theta = l.theta;
  a.thetadot = l.thetadot;
  a.best_key = l.key;
  a.status = l.status;
  a.trace_eef = l.trace_eef;
  a.trace_slots = l.trace_slots;
  a.slot_prev = e->d_slot_prev;
  a.jx = e->d_jx;
  a.tdscratch = e->d_td;
  a.hints = e->d_hints;
  a.pace = e->d_pace;
  a.mslab = e->d_mslab;
  a.dpar = l.dpar;
  a.state = l.state;
  a.plant = l.plant;
  a.dbg = l.dbg;
  a.layout = l.layout;
  a.n = l.n;
  a.H = e->H;
  a.nbasis = e->nbasis;
  a.index_base = l.index_base;
  a.nctrl = e->host.nctrl;
  a.nslot = e->host.nslot;
  a.seg_state = e->d_seg;
  a.seg = e->d_seg ? e->seg_steps : 0;
  a.seg_min_n = e->seg_min_n;
  std::memcpy(a.par, l.par, sizeof(a.par));
  if (l.key && l.reset_key) hipLaunchKernelGGL(fill_u64, dim3(1), dim3(1), 0, st, l.key, ~0ull);
  rollout_launch(e->wide, a, (const DevModel*)e->d_model, l.n, MPCR_N_DYN_LDS, st, e->seg_groups, e->seg_stream,
                 e->seg_event);
  HIPCHK(hipGetLastError());
  return MPCR_OK;
}

extern "C" int mpcr_set_two_wave_max_n(int n) { return rollout_set_wpc2_max_n(n); }

extern "C" int mpcr_engine_dispatches(const mpcr_engine* e, int n, int* out) {
  if (!e || !out) return fail(MPCR_EINVAL, "null argument");
  if (n < 0 || n > e->max_n) return fail(MPCR_EINVAL, "n=%d outside [0, max_n=%d]", n, e->max_n);
  RolloutArgs a;
  std::memset(&a, 0, sizeof(a));
  a.H = e->H;
  a.seg_state = e->d_seg;
  a.seg = e->d_seg ? e->seg_steps : 0;
  a.seg_min_n = e->seg_min_n;
  *out = rollout_dispatches(e->wide, a, n, e->seg_groups, e->seg_stream[0] != nullptr);
  return MPCR_OK;
}

extern "C" int mpcr_rollout_occupancy(int device, int* info) {
  if (!info) return fail(MPCR_EINVAL, "null argument");
  HIPCHK(hipSetDevice(device));
  HIPCHK(rollout_occupancy(info, MPCR_N_DYN_LDS));
  return MPCR_OK;
}

extern "C" int mpcr_rollout_cost(mpcr_engine* e, const float* input, int layout, int n, const double* q0,
                                 const float* w, const float* ptgt, const float* qtgt, float* cost4, float* theta,
                                 float* thetadot, uint64_t* best_key, int index_base, int* status, int flags,
                                 void* stream) {
  if (!e || !q0 || !w || !ptgt || !qtgt) return fail(MPCR_EINVAL, "null argument");
  if (n < 0 || n > e->max_n) return fail(MPCR_EINVAL, "n=%d outside [0, max_n=%d]", n, e->max_n);
  if (layout != MPCR_LAYOUT_XI && layout != MPCR_LAYOUT_THETADOT) return fail(MPCR_EINVAL, "bad layout %d", layout);
  if (n == 0) return MPCR_OK;  // an empty batch: input / cost4 may be null (a zero-size tensor's data pointer)
  if (!input || !cost4) return fail(MPCR_EINVAL, "null argument");
  HIPCHK(hipSetDevice(e->device));
  hipStream_t st = (hipStream_t)stream;
  auto* key = reinterpret_cast<unsigned long long*>(best_key);
  const int nc = e->host.nctrl;
  const size_t cols = layout == MPCR_LAYOUT_XI ? (size_t)nc * e->nbasis : (size_t)nc * e->H;
  Launch l;
  l.layout = layout;
  l.n = n;
  l.index_base = index_base;
  fill_par(l.par, nc, q0, w, ptgt, qtgt);
  if (flags & MPCR_F_DEVICE_PTRS) {
    l.in = input; l.cost4 = cost4; l.theta = theta; l.thetadot = thetadot; l.key = key; l.status = status;
    l.reset_key = (flags & MPCR_F_RESET_BEST) != 0;
    int rc = launch_rollout(e, l, st);
    if (rc) return rc;
    if (flags & MPCR_F_SYNC) HIPCHK(hipStreamSynchronize(st));
    return MPCR_OK;
  }
  HIPCHK(hipMemcpyAsync(e->d_in, input, sizeof(float) * n * cols, hipMemcpyHostToDevice, st));
  l.in = e->d_in; l.cost4 = e->d_cost; l.theta = theta ? e->d_theta : nullptr;
  l.thetadot = thetadot ? e->d_thetadot : nullptr; l.key = best_key ? e->d_key : nullptr;
  l.status = status ? e->d_status : nullptr; l.reset_key = true;
  int rc = launch_rollout(e, l, st);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(cost4, e->d_cost, sizeof(float) * 4 * n, hipMemcpyDeviceToHost, st));
  if (theta) HIPCHK(hipMemcpyAsync(theta, e->d_theta, sizeof(float) * n * nc * e->H, hipMemcpyDeviceToHost, st));
  if (thetadot)
    HIPCHK(hipMemcpyAsync(thetadot, e->d_thetadot, sizeof(float) * n * nc * e->H, hipMemcpyDeviceToHost, st));
  if (best_key) HIPCHK(hipMemcpyAsync(best_key, e->d_key, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  if (status) HIPCHK(hipMemcpyAsync(status, e->d_status, sizeof(int) * n, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return MPCR_OK;
}

extern "C" int mpcr_rollout_cost_dp(mpcr_engine* e, const float* input, int layout, int n, const float* params,
                                    float* cost4, float* theta, float* thetadot, uint64_t* best_key, int index_base,
                                    int* status, int flags, void* stream) {
  if (!e) return fail(MPCR_EINVAL, "null argument");
  if (n < 0 || n > e->max_n) return fail(MPCR_EINVAL, "n=%d outside [0, max_n=%d]", n, e->max_n);
  if (layout != MPCR_LAYOUT_XI && layout != MPCR_LAYOUT_THETADOT) return fail(MPCR_EINVAL, "bad layout %d", layout);
  if (n == 0) return MPCR_OK;  // an empty batch: the buffers may be null
  if (!input || !params || !cost4) return fail(MPCR_EINVAL, "null argument");
  HIPCHK(hipSetDevice(e->device));
  hipStream_t st = (hipStream_t)stream;
  Launch l;
  l.layout = layout; l.n = n; l.index_base = index_base; l.dpar = params;
  l.in = input; l.cost4 = cost4; l.theta = theta; l.thetadot = thetadot;
  l.key = reinterpret_cast<unsigned long long*>(best_key); l.status = status;
  l.reset_key = (flags & MPCR_F_RESET_BEST) != 0;
  int rc = launch_rollout(e, l, st);
  if (rc) return rc;
  if (flags & MPCR_F_SYNC) HIPCHK(hipStreamSynchronize(st));
  return MPCR_OK;
}

// ---------------------------------------------------------------------------
// closed-loop plant: one environment stepped by the same kernel (n = 1, H = 1,
// qvel[:nctrl] overridden like SBP/mpc_planner.py:179-180), state resident on
// the device between calls

struct mpcr_plant {
  mpcr_engine* e = nullptr;
  float* d_state = nullptr;  // ST_N floats (rollout.hip layout)
  float* d_in = nullptr;     // nctrl joint velocities
  float* d_cost = nullptr;   // unused cost4 of the single "candidate"
  float h_state[ST_N] = {};
};

extern "C" void mpcr_plant_free(mpcr_plant* p) {
  if (!p) return;
  (void)hipFree(p->d_state);
  (void)hipFree(p->d_in);
  (void)hipFree(p->d_cost);
  mpcr_engine_free(p->e);
  delete p;
}

extern "C" int mpcr_plant_create(const mpcr_model* m, int device, mpcr_plant** out) {
  if (!m || !out) return fail(MPCR_EINVAL, "null argument");
  const float pdot[1] = {0.f};
  auto* p = new mpcr_plant;
  int rc = mpcr_engine_create(m, device, 1, 1, pdot, 1, &p->e);
  if (rc) { delete p; return rc; }
  if (hipMalloc(&p->d_state, sizeof(float) * ST_N) != hipSuccess ||
      hipMalloc(&p->d_in, sizeof(float) * DX_NCTRL) != hipSuccess ||
      hipMalloc(&p->d_cost, sizeof(float) * 4) != hipSuccess) {
    mpcr_plant_free(p);
    return fail(MPCR_ENOMEM, "device allocation failed");
  }
  const mpcr_model_t& h = p->e->host;
  for (int i = 0; i < h.nq; i++) p->h_state[ST_QPOS + i] = (float)h.qpos_init[i];
  for (int i = 0; i < h.nv; i++) p->h_state[ST_QVEL + i] = (float)h.qvel_init[i];
  if (hipMemcpy(p->d_state, p->h_state, sizeof(float) * ST_N, hipMemcpyHostToDevice) != hipSuccess) {
    mpcr_plant_free(p);
    return fail(MPCR_EHIP, "state upload failed");
  }
  *out = p;
  return MPCR_OK;
}

extern "C" int mpcr_plant_set_state(mpcr_plant* p, const double* qpos, const double* qvel,
                                    const double* qacc_warmstart) {
  if (!p) return fail(MPCR_EINVAL, "null plant");
  HIPCHK(hipSetDevice(p->e->device));
  const mpcr_model_t& h = p->e->host;
  HIPCHK(hipMemcpy(p->h_state, p->d_state, sizeof(float) * ST_N, hipMemcpyDeviceToHost));
  if (qpos)
    for (int i = 0; i < h.nq; i++) p->h_state[ST_QPOS + i] = (float)qpos[i];
  if (qvel)
    for (int i = 0; i < h.nv; i++) p->h_state[ST_QVEL + i] = (float)qvel[i];
  if (qacc_warmstart)
    for (int i = 0; i < h.nv; i++) p->h_state[ST_QWS + i] = (float)qacc_warmstart[i];
  HIPCHK(hipMemcpy(p->d_state, p->h_state, sizeof(float) * ST_N, hipMemcpyHostToDevice));
  // a new state starts a new trajectory: the hull-climb starts the plant
  // keeps across steps (like a rollout's, and the oracle's) start over
  HIPCHK(hipMemset(p->e->d_hints, 0xff, sizeof(short) * 2 * (p->e->wide ? SmemW::NHINT : 1)));
  return MPCR_OK;
}

extern "C" int mpcr_plant_get_state(mpcr_plant* p, double* qpos, double* qvel, double* qacc, double* eef) {
  if (!p) return fail(MPCR_EINVAL, "null plant");
  HIPCHK(hipSetDevice(p->e->device));
  const mpcr_model_t& h = p->e->host;
  HIPCHK(hipMemcpy(p->h_state, p->d_state, sizeof(float) * ST_N, hipMemcpyDeviceToHost));
  if (qpos)
    for (int i = 0; i < h.nq; i++) qpos[i] = p->h_state[ST_QPOS + i];
  if (qvel)
    for (int i = 0; i < h.nv; i++) qvel[i] = p->h_state[ST_QVEL + i];
  if (qacc)
    for (int i = 0; i < h.nv; i++) qacc[i] = p->h_state[ST_QACC + i];
  if (eef)
    for (int i = 0; i < 7; i++) eef[i] = p->h_state[ST_EEF + i];
  return MPCR_OK;
}

// commit = 0: mj_forward (qacc and the eef pose of the current state, nothing
// advanced; qvel_ctrl ignored); commit = 1: mj_step with qvel[:nctrl] =
// qvel_ctrl (NULL keeps the current joint velocities)
extern "C" int mpcr_plant_step(mpcr_plant* p, const double* qvel_ctrl, int commit, void* stream) {
  if (!p) return fail(MPCR_EINVAL, "null plant");
  mpcr_engine* e = p->e;
  HIPCHK(hipSetDevice(e->device));
  hipStream_t st = (hipStream_t)stream;
  const int nc = e->host.nctrl;
  float v[DX_NCTRL] = {};
  if (!commit || !qvel_ctrl) {
    HIPCHK(hipMemcpyAsync(p->h_state, p->d_state, sizeof(float) * ST_N, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    for (int k = 0; k < nc; k++) v[k] = p->h_state[ST_QVEL + e->host.ctrl_dofadr[k]];
  } else {
    for (int k = 0; k < nc; k++) v[k] = (float)qvel_ctrl[k];
  }
  HIPCHK(hipMemcpyAsync(p->d_in, v, sizeof(float) * nc, hipMemcpyHostToDevice, st));
  Launch l;
  l.layout = MPCR_LAYOUT_THETADOT; l.n = 1; l.in = p->d_in; l.cost4 = p->d_cost;
  l.state = p->d_state; l.plant = commit ? 3 : 1;
  const double q0[DX_NCTRL] = {};
  const float w[3] = {0.f, 0.f, 0.f}, pt[3] = {0.f, 0.f, 0.f}, qt[4] = {1.f, 0.f, 0.f, 0.f};
  fill_par(l.par, nc, q0, w, pt, qt);
  int rc = launch_rollout(e, l, st);
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(st));
  return MPCR_OK;
}

// Debug/parity entry (not part of the stable ABI surface): one committed
// plant step (as mpcr_plant_step) that also copies the step's active
// contacts, constraint-row parameters, qacc_smooth and final qacc into
// dbg_host (mpcr_plant_dbg_size() floats; layout DBG_* of rollout.h, the
// oracle's oracle_step_debug writes the same).
extern "C" int mpcr_plant_dbg_size(void) { return DBG_N; }
extern "C" int mpcr_plant_step_debug(mpcr_plant* p, const double* qvel_ctrl, float* dbg_host, int mpr_pair) {
  if (!p || !qvel_ctrl || !dbg_host) return fail(MPCR_EINVAL, "bad debug step arguments");
  mpcr_engine* e = p->e;
  HIPCHK(hipSetDevice(e->device));
  const int nc = e->host.nctrl;
  float v[DX_NCTRL] = {};
  for (int k = 0; k < nc; k++) v[k] = (float)qvel_ctrl[k];
  float* d_dbg = nullptr;
  HIPCHK(hipMalloc(&d_dbg, sizeof(float) * DBG_N));
  HIPCHK(hipMemset(d_dbg, 0, sizeof(float) * DBG_N));
  const float pf = (float)mpr_pair;  // the pair whose MPR the kernel traces (DBG_MPR), -1: none
  HIPCHK(hipMemcpy(d_dbg + DBG_MPR, &pf, sizeof(float), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(p->d_in, v, sizeof(float) * nc, hipMemcpyHostToDevice));
  Launch l;
  l.layout = MPCR_LAYOUT_THETADOT; l.n = 1; l.in = p->d_in; l.cost4 = p->d_cost;
  l.state = p->d_state; l.plant = 3; l.dbg = d_dbg;
  const double q0[DX_NCTRL] = {};
  const float w[3] = {0.f, 0.f, 0.f}, pt[3] = {0.f, 0.f, 0.f}, qt[4] = {1.f, 0.f, 0.f, 0.f};
  fill_par(l.par, nc, q0, w, pt, qt);
  int rc = launch_rollout(e, l, 0);
  if (rc) { (void)hipFree(d_dbg); return rc; }
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(dbg_host, d_dbg, sizeof(float) * DBG_N, hipMemcpyDeviceToHost));
  HIPCHK(hipFree(d_dbg));
  return MPCR_OK;
}

// Debug/parity entry (not part of the stable ABI surface): host pointers,
// also returns the per-step eef pose (n x H x 7) and masked slot distances
// (n x H x nslot).
extern "C" int mpcr_rollout_trace(mpcr_engine* e, const float* input, int layout, int n, const double* q0,
                                  const float* w, const float* ptgt, const float* qtgt, float* cost4, float* theta,
                                  float* eef, float* slots) {
  if (!e || !input || !cost4 || n <= 0 || n > e->max_n) return fail(MPCR_EINVAL, "bad trace arguments");
  HIPCHK(hipSetDevice(e->device));
  const int nc = e->host.nctrl;
  const size_t cols = layout == MPCR_LAYOUT_XI ? (size_t)nc * e->nbasis : (size_t)nc * e->H;
  float *d_eef = nullptr, *d_slots = nullptr;
  const int nslot = e->host.nslot > 0 ? e->host.nslot : 1;
  HIPCHK(hipMalloc(&d_eef, sizeof(float) * n * e->H * 7));
  HIPCHK(hipMalloc(&d_slots, sizeof(float) * n * e->H * nslot));
  HIPCHK(hipMemcpy(e->d_in, input, sizeof(float) * n * cols, hipMemcpyHostToDevice));
  Launch l;
  l.layout = layout; l.n = n; l.in = e->d_in; l.cost4 = e->d_cost; l.theta = e->d_theta; l.status = e->d_status;
  l.trace_eef = d_eef; l.trace_slots = d_slots;
  fill_par(l.par, nc, q0, w, ptgt, qtgt);
  int rc = launch_rollout(e, l, nullptr);
  if (rc == 0) {
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(cost4, e->d_cost, sizeof(float) * 4 * n, hipMemcpyDeviceToHost));
    if (theta) HIPCHK(hipMemcpy(theta, e->d_theta, sizeof(float) * n * nc * e->H, hipMemcpyDeviceToHost));
    if (eef) HIPCHK(hipMemcpy(eef, d_eef, sizeof(float) * n * e->H * 7, hipMemcpyDeviceToHost));
    if (slots) HIPCHK(hipMemcpy(slots, d_slots, sizeof(float) * n * e->H * nslot, hipMemcpyDeviceToHost));
  }
  (void)hipFree(d_eef);
  (void)hipFree(d_slots);
  return rc;
}

#ifdef MPCR_PROFILE
// diagnostic build only: per-phase s_memtime cycles summed over all waves
extern "C" int mpcr_rollout_profile(mpcr_engine* e, const float* input, int layout, int n, const double* q0,
                                    const float* w, const float* ptgt, const float* qtgt,
                                    unsigned long long* phases16 /* 64 slots: wave 0, wave 1 (WPC = 2) */) {
  HIPCHK(hipSetDevice(e->device));
  const int nc = e->host.nctrl;
  const size_t cols = layout == MPCR_LAYOUT_XI ? (size_t)nc * e->nbasis : (size_t)nc * e->H;
  unsigned long long* d_prof = nullptr;
  HIPCHK(hipMalloc(&d_prof, 64 * sizeof(unsigned long long)));
  HIPCHK(hipMemset(d_prof, 0, 64 * sizeof(unsigned long long)));
  e->dev.prof = d_prof;  // wave-level counters for this launch only
  HIPCHK(hipMemcpy(e->d_model, &e->dev, sizeof(DevModel), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(e->d_in, input, sizeof(float) * n * cols, hipMemcpyHostToDevice));
  RolloutArgs a;
  std::memset(&a, 0, sizeof(a));
  a.m = e->d_model; a.input = e->d_in; a.pdot = e->d_pdot; a.cost4 = e->d_cost; a.prof = d_prof;
  a.slot_prev = e->d_slot_prev;
  a.jx = e->d_jx;
  a.tdscratch = e->d_td;
  a.hints = e->d_hints;
  a.pace = e->d_pace;
  a.mslab = e->d_mslab;
  a.layout = layout; a.n = n; a.H = e->H; a.nbasis = e->nbasis;
  fill_par(a.par, nc, q0, w, ptgt, qtgt);
  rollout_launch(e->wide, a, (const DevModel*)e->d_model, n, MPCR_N_DYN_LDS, nullptr);
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(phases16, d_prof, 64 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  e->dev.prof = nullptr;
  HIPCHK(hipMemcpy(e->d_model, &e->dev, sizeof(DevModel), hipMemcpyHostToDevice));
  (void)hipFree(d_prof);
  return MPCR_OK;
}
#endif

#ifdef MPCR_WAVETIME
// diagnostic build only: per wave (start, end) on the 100 MHz clock, shader
// cycles, (XCC_ID << 32 | HW_ID) -- 4 u64 per candidate; then per candidate
// (line-search passes << 32 | Newton iterations, convex flush chunks)
extern "C" int mpcr_rollout_wavetime(mpcr_engine* e, const float* input, int layout, int n, const double* q0,
                                     const float* w, const float* ptgt, const float* qtgt, unsigned long long* out) {
  HIPCHK(hipSetDevice(e->device));
  const int nc = e->host.nctrl;
  const size_t cols = layout == MPCR_LAYOUT_XI ? (size_t)nc * e->nbasis : (size_t)nc * e->H;
  unsigned long long* d_prof = nullptr;
  HIPCHK(hipMalloc(&d_prof, 6 * (size_t)n * sizeof(unsigned long long)));
  HIPCHK(hipMemset(d_prof, 0, 6 * (size_t)n * sizeof(unsigned long long)));
  HIPCHK(hipMemcpy(e->d_in, input, sizeof(float) * n * cols, hipMemcpyHostToDevice));
  RolloutArgs a;
  std::memset(&a, 0, sizeof(a));
  a.m = e->d_model; a.input = e->d_in; a.pdot = e->d_pdot; a.cost4 = e->d_cost; a.prof = d_prof;
  a.slot_prev = e->d_slot_prev;
  a.jx = e->d_jx;
  a.tdscratch = e->d_td;
  a.hints = e->d_hints;
  a.pace = e->d_pace;
  a.mslab = e->d_mslab;
  a.layout = layout; a.n = n; a.H = e->H; a.nbasis = e->nbasis;
  fill_par(a.par, nc, q0, w, ptgt, qtgt);
  rollout_launch(e->wide, a, (const DevModel*)e->d_model, n, MPCR_N_DYN_LDS, nullptr);
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(out, d_prof, 6 * (size_t)n * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  (void)hipFree(d_prof);
  return MPCR_OK;
}
#endif

extern "C" void mpcr_best_key_decode(uint64_t key, int* idx, float* cost) {
  uint32_t hi = (uint32_t)(key >> 32);
  if (idx) *idx = (int)(uint32_t)(key & 0xffffffffu);
  if (cost) {
    if (hi == 0u) {
      *cost = NAN;
    } else {
      uint32_t u = (hi & 0x80000000u) ? (hi & 0x7fffffffu) : ~hi;
      float f;
      std::memcpy(&f, &u, 4);
      *cost = f;
    }
  }
}

extern "C" int mpcr_argmin(mpcr_engine* e, const float* cost, int stride, int n, int index_base, uint64_t* key_out,
                           int* idx_out, float* val_out, int flags, void* stream) {
  if (!e || !cost || n <= 0 || stride <= 0) return fail(MPCR_EINVAL, "bad argmin arguments");
  HIPCHK(hipSetDevice(e->device));
  hipStream_t st = (hipStream_t)stream;
  const float* dcost = cost;
  if (!(flags & MPCR_F_DEVICE_PTRS)) {
    if (n > e->max_n || stride > 4) return fail(MPCR_EINVAL, "host argmin limited to max_n x 4");
    HIPCHK(hipMemcpyAsync(e->d_cost, cost, sizeof(float) * (size_t)n * stride, hipMemcpyHostToDevice, st));
    dcost = e->d_cost;
  }
  unsigned long long* key = (flags & MPCR_F_DEVICE_PTRS) && key_out ? reinterpret_cast<unsigned long long*>(key_out)
                                                                    : e->d_key;
  hipLaunchKernelGGL(fill_u64, dim3(1), dim3(1), 0, st, key, ~0ull);
  int blocks = (n + 255) / 256;
  blocks = blocks > 1024 ? 1024 : blocks;
  hipLaunchKernelGGL(argmin_kernel, dim3(blocks), dim3(256), 0, st, dcost, stride, n, index_base, key);
  HIPCHK(hipGetLastError());
  if (idx_out || val_out || (key_out && !(flags & MPCR_F_DEVICE_PTRS))) {
    uint64_t k;
    HIPCHK(hipMemcpyAsync(&k, key, sizeof(k), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    mpcr_best_key_decode(k, idx_out, val_out);
    if (key_out && !(flags & MPCR_F_DEVICE_PTRS)) *key_out = k;
  } else if (flags & MPCR_F_SYNC) {
    HIPCHK(hipStreamSynchronize(st));
  }
  return MPCR_OK;
}

extern "C" int mpcr_topk(mpcr_engine* e, const float* cost, int stride, int n, int k, int* idx_out, int flags,
                         void* stream) {
  if (!e || !cost || !idx_out || stride <= 0 || n < 0) return fail(MPCR_EINVAL, "bad topk arguments");
  if (k < 0 || k > n || k > TOPK_MAX) return fail(MPCR_EINVAL, "k=%d outside [0, min(n=%d, %d)]", k, n, TOPK_MAX);
  if (k == 0) return MPCR_OK;
  HIPCHK(hipSetDevice(e->device));
  hipStream_t st = (hipStream_t)stream;
  if (flags & MPCR_F_DEVICE_PTRS) {
    hipLaunchKernelGGL(topk_kernel, dim3(1), dim3(1024), 0, st, cost, stride, n, k, idx_out);
    HIPCHK(hipGetLastError());
    if (flags & MPCR_F_SYNC) HIPCHK(hipStreamSynchronize(st));
    return MPCR_OK;
  }
  if (n > e->max_n || stride > 4) return fail(MPCR_EINVAL, "host topk limited to max_n x 4");
  HIPCHK(hipMemcpyAsync(e->d_cost, cost, sizeof(float) * (size_t)n * stride, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(topk_kernel, dim3(1), dim3(1024), 0, st, e->d_cost, stride, n, k, e->d_idx);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(idx_out, e->d_idx, sizeof(int) * k, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return MPCR_OK;
}

// ---------------------------------------------------------------------------
// CEM context (cem.hip kernels)

struct mpcr_cem {
  int device = 0, nd = 0, H = 0, max_n = 0;
  float* d_X = nullptr;    // 3 x H x 12: Pdot, Pddot, P
  float* d_QT = nullptr;   // LD x LD
  float* d_QbT = nullptr;  // 5nd x LD
  float* d_LT = nullptr;   // LD x LD Cholesky factor (transposed, padded)
  bool factored = false;
};

// get_Q_inv (SBP/mjx_planner.py:166-172 as restated by oracle/cem_np.q_inv):
// fp32 Gram blocks of kron(I, [X; -X]) promoted to fp64, fp64 KKT inverse.
static bool kkt_inverse(int nd, int H, const float* P, const float* Pd, const float* Pdd, std::vector<double>& Kinv) {
  const int nb = PJ_NB, nv = nd * nb, ne = 5 * nd, NK = nv + ne;
  std::vector<double> K((size_t)NK * NK, 0.0);
  const float* mats[3] = {Pd, Pdd, P};
  for (int a = 0; a < nb; a++)
    for (int b = 0; b < nb; b++) {
      double g = 0.0;
      for (int k = 0; k < 3; k++) {
        float s = 0.f;  // fp32 Gram entry over the 2H rows of [X; -X]
        for (int t = 0; t < H; t++) s += mats[k][t * nb + a] * mats[k][t * nb + b];
        for (int t = 0; t < H; t++) s += (-mats[k][t * nb + a]) * (-mats[k][t * nb + b]);
        g += (double)s;
      }
      for (int j = 0; j < nd; j++) K[(size_t)(j * nb + a) * NK + j * nb + b] = g + (a == b ? 1.0 : 0.0);
    }
  for (int j = 0; j < nd; j++)
    for (int c = 0; c < nb; c++) {
      const double rows[5] = {P[c], Pd[c], Pdd[c], Pd[(H - 1) * nb + c], Pdd[(H - 1) * nb + c]};
      for (int m = 0; m < 5; m++) {
        K[(size_t)(nv + j * 5 + m) * NK + j * nb + c] = rows[m];
        K[(size_t)(j * nb + c) * NK + nv + j * 5 + m] = rows[m];
      }
    }
  // Gauss-Jordan with partial pivoting
  Kinv.assign((size_t)NK * NK, 0.0);
  for (int i = 0; i < NK; i++) Kinv[(size_t)i * NK + i] = 1.0;
  for (int c = 0; c < NK; c++) {
    int piv = c;
    for (int r = c + 1; r < NK; r++)
      if (std::fabs(K[(size_t)r * NK + c]) > std::fabs(K[(size_t)piv * NK + c])) piv = r;
    if (K[(size_t)piv * NK + c] == 0.0) return false;
    if (piv != c)
      for (int q = 0; q < NK; q++) {
        std::swap(K[(size_t)c * NK + q], K[(size_t)piv * NK + q]);
        std::swap(Kinv[(size_t)c * NK + q], Kinv[(size_t)piv * NK + q]);
      }
    const double inv = 1.0 / K[(size_t)c * NK + c];
    for (int q = 0; q < NK; q++) { K[(size_t)c * NK + q] *= inv; Kinv[(size_t)c * NK + q] *= inv; }
    for (int r = 0; r < NK; r++) {
      if (r == c) continue;
      const double f = K[(size_t)r * NK + c];
      if (f == 0.0) continue;
      for (int q = 0; q < NK; q++) {
        K[(size_t)r * NK + q] -= f * K[(size_t)c * NK + q];
        Kinv[(size_t)r * NK + q] -= f * Kinv[(size_t)c * NK + q];
      }
    }
  }
  return true;
}

extern "C" int mpcr_cem_create(int device, int num_dof, int horizon, int nbasis, const double* P, const double* Pdot,
                               const double* Pddot, const double* qinv, int max_n, mpcr_cem** out) {
  if (!out || !P || !Pdot || !Pddot || max_n <= 0 || horizon < 2) return fail(MPCR_EINVAL, "bad cem arguments");
  if (nbasis != PJ_NB) return fail(MPCR_EINVAL, "nbasis=%d: the CEM kernels are built for order-10 (11)", nbasis);
  if (num_dof < 1 || num_dof > PJ_MAXD) return fail(MPCR_EINVAL, "num_dof=%d outside [1, %d]", num_dof, PJ_MAXD);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(MPCR_ENODEV, "no HIP device");
  if (device < 0 || device >= ndev) return fail(MPCR_ENODEV, "device %d out of range (%d)", device, ndev);
  HIPCHK(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(MPCR_ENODEV, "device %d is %s; libmpcr is built for gfx950 only", device, prop.gcnArchName);
  const int nd = num_dof, H = horizon, nb = PJ_NB, nv = nd * nb, ne = 5 * nd, NK = nv + ne, LD = nd * PJ_BLK;
  {
    // sample_project_kernel stages the constraint rows X (3 x H x 12) and the
    // candidates' rows in LDS (mpcr_cem_sample_project): refuse a horizon
    // whose image exceeds the device's per-workgroup LDS
    const int cpw = PJ_CPW_LARGE > PJ_CPW_SMALL ? PJ_CPW_LARGE : PJ_CPW_SMALL;
    const size_t lds = sizeof(float) * (cpw * (nd * PJ_BLK + 4) + 3 * (size_t)H * PJ_BLK);
    if (lds > prop.sharedMemPerBlock)
      return fail(MPCR_EINVAL, "horizon=%d: the projection kernel's LDS image (%zu B) exceeds the device's %zu B per "
                  "workgroup", H, lds, (size_t)prop.sharedMemPerBlock);
  }
  std::vector<float> Pf((size_t)H * nb), Pdf((size_t)H * nb), Pddf((size_t)H * nb);
  for (int i = 0; i < H * nb; i++) { Pf[i] = (float)P[i]; Pdf[i] = (float)Pdot[i]; Pddf[i] = (float)Pddot[i]; }
  std::vector<double> Kinv;
  if (qinv) {
    Kinv.assign(qinv, qinv + (size_t)NK * NK);
  } else if (!kkt_inverse(nd, H, Pf.data(), Pdf.data(), Pddf.data(), Kinv)) {
    return fail(MPCR_EINVAL, "singular KKT matrix");
  }
  std::vector<float> X((size_t)3 * H * PJ_BLK, 0.f), QT((size_t)LD * LD, 0.f), QbT((size_t)ne * LD, 0.f);
  const float* mats[3] = {Pdf.data(), Pddf.data(), Pf.data()};
  for (int k = 0; k < 3; k++)
    for (int t = 0; t < H; t++)
      for (int c = 0; c < nb; c++) X[((size_t)k * H + t) * PJ_BLK + c] = mats[k][t * nb + c];
  auto pad = [&](int i) { return (i / nb) * PJ_BLK + i % nb; };
  for (int r = 0; r < nv; r++) {
    for (int c = 0; c < nv; c++) QT[(size_t)pad(c) * LD + pad(r)] = (float)Kinv[(size_t)r * NK + c];
    for (int m = 0; m < ne; m++) QbT[(size_t)m * LD + pad(r)] = (float)Kinv[(size_t)r * NK + nv + m];
  }
  auto* c = new mpcr_cem;
  c->device = device;
  c->nd = nd;
  c->H = H;
  c->max_n = max_n;
  if (hipMalloc(&c->d_X, sizeof(float) * X.size()) != hipSuccess ||
      hipMalloc(&c->d_QT, sizeof(float) * QT.size()) != hipSuccess ||
      hipMalloc(&c->d_QbT, sizeof(float) * QbT.size()) != hipSuccess ||
      hipMalloc(&c->d_LT, sizeof(float) * (size_t)LD * LD) != hipSuccess) {
    mpcr_cem_free(c);
    return fail(MPCR_ENOMEM, "device allocation failed");
  }
  if (hipMemcpy(c->d_X, X.data(), sizeof(float) * X.size(), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(c->d_QT, QT.data(), sizeof(float) * QT.size(), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(c->d_QbT, QbT.data(), sizeof(float) * QbT.size(), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(c->d_LT, 0, sizeof(float) * (size_t)LD * LD) != hipSuccess) {
    mpcr_cem_free(c);
    return fail(MPCR_EHIP, "table upload failed");
  }
  *out = c;
  return MPCR_OK;
}

extern "C" void mpcr_cem_free(mpcr_cem* c) {
  if (!c) return;
  (void)hipFree(c->d_X);
  (void)hipFree(c->d_QT);
  (void)hipFree(c->d_QbT);
  (void)hipFree(c->d_LT);
  delete c;
}

extern "C" int mpcr_cem_factor(mpcr_cem* c, const float* cov, float reg, int flags, void* stream) {
  if (!c || !cov) return fail(MPCR_EINVAL, "null argument");
  if (!(flags & MPCR_F_DEVICE_PTRS)) return fail(MPCR_EINVAL, "mpcr_cem_factor takes device pointers");
  HIPCHK(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(cholesky_kernel, dim3(1), dim3(256), 0, st, cov, c->nd, reg, c->d_LT);
  HIPCHK(hipGetLastError());
  c->factored = true;
  if (flags & MPCR_F_SYNC) HIPCHK(hipStreamSynchronize(st));
  return MPCR_OK;
}

extern "C" int mpcr_cem_sample_project(mpcr_cem* c, int n, const float* mean, uint64_t seed, uint64_t counter,
                                       int index_base, const float* xi_in, float* xi_samples, const float* b_eq, int beq_stride,
                                       int maxiter, const float* bounds, float rho, float* xi_out, int flags,
                                       void* stream) {
  if (!c || !xi_out) return fail(MPCR_EINVAL, "null argument");
  if (!(flags & MPCR_F_DEVICE_PTRS)) return fail(MPCR_EINVAL, "mpcr_cem_sample_project takes device pointers");
  if (n < 0 || n > c->max_n) return fail(MPCR_EINVAL, "n=%d outside [0, max_n=%d]", n, c->max_n);
  if (!mean && !xi_in) return fail(MPCR_EINVAL, "need mean (sampling) or xi_in");
  if (mean && !c->factored) return fail(MPCR_EINVAL, "sampling before mpcr_cem_factor");
  if (maxiter < 0 || (maxiter > 0 && (!b_eq || !bounds || beq_stride < 0)))
    return fail(MPCR_EINVAL, "projection needs b_eq, bounds and maxiter >= 0");
  if (n == 0) return MPCR_OK;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  ProjArgs a;
  std::memset(&a, 0, sizeof(a));
  a.xi_in = xi_in;
  a.mean = mean;
  a.L = c->d_LT;
  a.xi_samples = xi_samples;
  a.beq = b_eq;
  a.xi_out = xi_out;
  a.X = c->d_X;
  a.QT = c->d_QT;
  a.QbT = c->d_QbT;
  a.seed = seed;
  a.counter = counter;
  a.index_base = index_base;
  a.n = n;
  a.nd = c->nd;
  a.H = c->H;
  a.maxiter = maxiter;
  a.beq_stride = beq_stride;
  for (int k = 0; k < 3; k++) a.bound[k] = bounds ? bounds[k] : 0.f;
  a.rho = rho;
  // the candidates' padded rows and the constraint rows X (3 x H x 12) in LDS
  const int cpw = n >= PJ_CPW_SWITCH ? PJ_CPW_LARGE : PJ_CPW_SMALL;
  const size_t lds = sizeof(float) * (cpw * (c->nd * PJ_BLK + 4) + 3 * (size_t)c->H * PJ_BLK);
  if (cpw == PJ_CPW_LARGE)
    hipLaunchKernelGGL(sample_project_kernel<PJ_CPW_LARGE>, dim3((n + cpw - 1) / cpw), dim3(64 * c->nd), lds, st, a);
  else
    hipLaunchKernelGGL(sample_project_kernel<PJ_CPW_SMALL>, dim3((n + cpw - 1) / cpw), dim3(64 * c->nd), lds, st, a);
  HIPCHK(hipGetLastError());
  if (flags & MPCR_F_SYNC) HIPCHK(hipStreamSynchronize(st));
  return MPCR_OK;
}

extern "C" int mpcr_project(mpcr_cem* c, const float* xi, const float* b_eq, int beq_stride, int n, int maxiter,
                            const float* bounds, float rho, float* xi_out, int flags, void* stream) {
  if (!xi) return fail(MPCR_EINVAL, "null xi");
  return mpcr_cem_sample_project(c, n, nullptr, 0, 0, 0, xi, nullptr, b_eq, beq_stride, maxiter, bounds, rho, xi_out,
                                 flags, stream);
}

extern "C" int mpcr_cem_update(mpcr_cem* c, const float* xi, int n, const float* cost, int stride,
                               const int* elite_idx, int k, float lamda, float alpha_mean, float alpha_cov, float reg,
                               float* mean, float* cov, int flags, void* stream) {
  if (!c || !xi || !cost || !elite_idx || !mean || !cov || stride <= 0) return fail(MPCR_EINVAL, "null argument");
  if (!(flags & MPCR_F_DEVICE_PTRS)) return fail(MPCR_EINVAL, "mpcr_cem_update takes device pointers");
  if (k <= 0 || k > n || k > TOPK_MAX) return fail(MPCR_EINVAL, "k=%d outside [1, min(n=%d, %d)]", k, n, TOPK_MAX);
  HIPCHK(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(cem_update_kernel, dim3(1), dim3(1024), 0, st, xi, c->nd * PJ_NB, cost, stride, elite_idx, k,
                     lamda, alpha_mean, alpha_cov, reg, mean, cov);
  HIPCHK(hipGetLastError());
  if (flags & MPCR_F_SYNC) HIPCHK(hipStreamSynchronize(st));
  return MPCR_OK;
}

#include "comm.hip"
