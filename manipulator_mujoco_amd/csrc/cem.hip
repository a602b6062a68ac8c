// cem.hip — the CEM distribution step around the rollout (SURVEY.md §8a
// A10, A12, A13; §8f-1/2): MVN sampling, the ADMM projection filter, top-E
// elite selection and the weighted mean/covariance update.  Included by
// engine.hip after the error helpers; the host entry points are at the end.
//
// Reference semantics (SBP/mjx_planner.py, restated as in oracle/cem_np.py):
//   compute_xi_samples  :312-316   xi = mean + z L^T, L = chol(cov + 0.003 I)
//   compute_projection  :181-231   one ADMM iteration (rho, slacks, multipliers)
//   compute_projection_filter :234-249  maxiter unrolled iterations
//   compute_ellite_samples    :305-310  stable argsort, first E
//   compute_mean_cov / comp_prod :318-335
//
// Projection algebra.  For A_k = kron(I, [X_k; -X_k]) and v = X_k p (per
// joint), the reference's slack s = max(b - A p, 0), residual
// res = A p - b + s = max(A p - b, 0) and A_k^T (b - s) only depend on v:
//   A_k^T (b - s_k)  = sum_t X_k[t,:] * (max(b+v,0) - max(b-v,0))
//   A_k^T res_k      = sum_t X_k[t,:] * (max(v-b,0) - max(-v-b,0))
// so a thread owning (candidate, joint) keeps only p, xi, sum_k lambda_k and
// the next iteration's slack term (4 x 11 registers): nothing of size H is
// stored, and the dense 12H x 66 GEMMs become 3 x H x 11 row dots + two
// 11-wide axpys per row.  The KKT solve needs the candidate's whole
// right-hand side, exchanged through LDS.

namespace mpcr {

constexpr int PJ_NB = 11;    // order-10 Bernstein basis (the planner's)
constexpr int PJ_BLK = 12;   // per-joint block, padded (48-byte aligned rows)
constexpr int PJ_MAXD = 8;   // joints (waves per workgroup)
constexpr int TOPK_MAX = 4096;
constexpr int PJ_RG = 4;     // projection rows per load group (interleaved dot chains)
// candidates per workgroup (and per wave) of the projection kernel, chosen
// per launch: 16 below 8192 candidates, 32 from there (10-iteration
// projection, H = 50: 4096 -> 0.130 / 0.172 ms, 8192 -> 0.249 / 0.181 ms for
// 16 / 32; 8 gave 0.199 / 0.384 ms)
constexpr int PJ_CPW_SMALL = 16, PJ_CPW_LARGE = 32, PJ_CPW_SWITCH = 8192;

struct ProjArgs {
  const float* xi_in;     // n x nv (read when mean == nullptr)
  const float* mean;      // nv: sample mode (xi = mean + z L^T)
  const float* L;         // nd*12 x nd*12 padded lower Cholesky factor (sample mode)
  float* xi_samples;      // n x nv out (sample mode, nullable)
  const float* beq;       // n x 5nd, row stride beq_stride (0 = one shared row)
  float* xi_out;          // n x nv
  const float* X;         // 3 x H x 12: Pdot, Pddot, P rows (zero padded)
  const float* QT;        // nd*12 x nd*12: QT[c][r] = Qinv[r][c] (padded, zero pads)
  const float* QbT;       // 5nd x nd*12:   QbT[m][r] = Qinv[r][nv + m]
  unsigned long long seed, counter;
  int n, nd, H, maxiter, beq_stride;
  int index_base;         // global index of candidate 0 (Philox counter word 0)
  float bound[3];         // v_max, a_max, p_max
  float rho;
};

// Philox4x32-10 (Salmon et al., SC'11), counter-based: each (candidate,
// joint, block) draws its own 4 words, so samples do not depend on the
// launch shape.
__device__ __forceinline__ void philox4(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; r++) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c[0]), lo0 = 0xD2511F53u * c[0];
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c[2]), lo1 = 0xCD9E8D57u * c[2];
    const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}

// Box-Muller on two words: u1 in (0, 1], u2 in [0, 1)
__device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, float& z0, float& z1) {
  const float u1 = ((float)a + 1.0f) * 2.3283064365386963e-10f;
  const float u2 = (float)b * 2.3283064365386963e-10f;
  const float r = sqrtf(-2.0f * logf(fminf(u1, 1.0f)));
  float s, c;
  sincosf(6.283185307179586f * u2, &s, &c);
  z0 = r * c;
  z1 = r * s;
}

// One workgroup = PJ_CPW candidates x nd waves; wave j owns joint j's 11
// coefficients of each of its candidates, and lane = candidate + PJ_CPW x
// part: the PJ_NP lanes of a candidate split the 3H constraint rows of each
// ADMM iteration and add their partial sums with two lane swaps.  Few
// candidates per workgroup spread a batch over every CU (64 candidates per
// workgroup left 3 of 4 CUs idle at 4096), and the split shortens each
// lane's chain of dependent row updates (the loop ran at ~10 cycles an
// instruction with one wave per SIMD).  The KKT solve is per candidate and
// repeated by its parts.
template <int PJ_CPW>
__global__ void __launch_bounds__(64 * PJ_MAXD) sample_project_kernel(ProjArgs a) {
  constexpr int PJ_NP = 64 / PJ_CPW;  // row parts: the lanes of one candidate
  extern __shared__ float pj_smem[];
  const int nd = a.nd, NV = nd * PJ_NB, RS = nd * PJ_BLK + 4;  // LDS row stride: conflict-free b128
  const int lane = threadIdx.x & 63;
  const int j = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform joint
  const int cl = lane & (PJ_CPW - 1), part = lane / PJ_CPW;  // candidate in the workgroup, row part
  const int cand = blockIdx.x * PJ_CPW + cl;
  const bool live = cand < a.n;
  float* row = pj_smem + cl * RS;  // this candidate's padded vector (rhs / z)
  const int jb = j * PJ_BLK;
  // the constraint rows X (identical for every joint, candidate and ADMM
  // iteration) in LDS
  float* const Xs = pj_smem + PJ_CPW * RS;
  for (int i = threadIdx.x; i < 3 * a.H * PJ_BLK; i += blockDim.x) Xs[i] = a.X[i];
  __syncthreads();

  float xi[PJ_NB];
  if (a.mean) {
    // z for this (candidate, joint): 3 Philox blocks -> 12 normals (11 used)
    float z[PJ_BLK];
#pragma unroll
    for (int q = 0; q < 3; q++) {
      uint32_t c[4] = {(uint32_t)(cand + a.index_base), (uint32_t)(j * 3 + q), (uint32_t)a.counter, (uint32_t)(a.counter >> 32)};
      philox4(c, (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
      box_muller(c[0], c[1], z[4 * q + 0], z[4 * q + 1]);
      box_muller(c[2], c[3], z[4 * q + 2], z[4 * q + 3]);
    }
    z[PJ_NB] = 0.f;
    if (part == 0) {
#pragma unroll
      for (int c = 0; c < PJ_BLK; c++) row[jb + c] = z[c];
    }
    __syncthreads();
    // xi[r] = mean[r] + sum_{c <= r} L[r][c] z[c]; L is stored transposed
    // (LT[c][r]) so the 11 coefficients of one c are contiguous and uniform.
    const int LD = nd * PJ_BLK;
#pragma unroll
    for (int r = 0; r < PJ_NB; r++) xi[r] = a.mean[j * PJ_NB + r];
    for (int j2 = 0; j2 <= j; j2++) {
      for (int c = 0; c < PJ_NB; c++) {
        const float zc = row[j2 * PJ_BLK + c];
        const float* lt = a.L + (size_t)(j2 * PJ_BLK + c) * LD + jb;
#pragma unroll
        for (int r = 0; r < PJ_NB; r++) xi[r] = fmaf(lt[r], zc, xi[r]);
      }
    }
    __syncthreads();  // row[] is reused for the right-hand side below
  } else {
#pragma unroll
    for (int r = 0; r < PJ_NB; r++) xi[r] = live ? a.xi_in[(size_t)cand * NV + j * PJ_NB + r] : 0.f;
  }

  float p[PJ_NB];
#pragma unroll
  for (int r = 0; r < PJ_NB; r++) p[r] = xi[r];
  if (a.maxiter > 0) {
    // constant part of the KKT solve: Qinv[rows, nv:] @ b_eq
    float qb[PJ_NB];
#pragma unroll
    for (int r = 0; r < PJ_NB; r++) qb[r] = 0.f;
    const float* be = a.beq + (live ? (size_t)cand * a.beq_stride : 0);
    for (int m = 0; m < 5 * nd; m++) {
      const float bm = be[m];
      const float* qt = a.QbT + (size_t)m * nd * PJ_BLK + jb;
#pragma unroll
      for (int r = 0; r < PJ_NB; r++) qb[r] = fmaf(qt[r], bm, qb[r]);
    }
    float lam[PJ_NB], sl[PJ_NB];  // sum_k lambda_k; sum_k A_k^T (b - s_k)
#pragma unroll
    for (int r = 0; r < PJ_NB; r++) lam[r] = sl[r] = 0.f;
    const int LD = nd * PJ_BLK;
    // the 3H rows of each constraint family fall into PJ_NR = 4 fixed ranges
    // whatever the layout, summed in one tree ((r0 + r1) + (r2 + r3)): a
    // part of PJ_NP = 4 lanes holds one range, of PJ_NP = 2 two (their sum
    // first), so a candidate's projection is bitwise the same at 16 and at
    // 32 candidates per workgroup -- i.e. independent of the batch size
    // (the sharded planner's ranks then reproduce one GPU at C5's 8192)
    constexpr int PJ_NR = 4, PJ_RPL = PJ_NR / PJ_NP;
    static_assert(PJ_NR % PJ_NP == 0, "row ranges per part");
    for (int it = 0; it < a.maxiter; it++) {
      // -lincost = lam + rho xi + rho sum_k A_k^T (b - s_k)  (every part holds
      // the same values; part 0 writes them)
      if (part == 0) {
#pragma unroll
        for (int r = 0; r < PJ_NB; r++) row[jb + r] = lam[r] + a.rho * xi[r] + a.rho * sl[r];
        row[jb + PJ_NB] = 0.f;
      }
      __syncthreads();
      // primal = Qinv[rows, :nv] @ rhs + qb  (QT rows are wave-uniform)
#pragma unroll
      for (int r = 0; r < PJ_NB; r++) p[r] = qb[r];
      for (int c = 0; c < LD; c += 4) {
        const float4 rv = *reinterpret_cast<const float4*>(row + c);
        const float* q0 = a.QT + (size_t)c * LD + jb;
#pragma unroll
        for (int r = 0; r < PJ_NB; r++) {
          p[r] = fmaf(q0[r], rv.x, p[r]);
          p[r] = fmaf(q0[LD + r], rv.y, p[r]);
          p[r] = fmaf(q0[2 * LD + r], rv.z, p[r]);
          p[r] = fmaf(q0[3 * LD + r], rv.w, p[r]);
        }
      }
      __syncthreads();  // everyone has read row[] before it is rewritten
      // slacks, residuals, multipliers for Pdot (v), Pddot (a), P (p): this
      // part's rows, then the parts' sums
      float dl[PJ_NB];
#pragma unroll
      for (int r = 0; r < PJ_NB; r++) dl[r] = sl[r] = 0.f;
#pragma unroll
      for (int rq = 0; rq < PJ_RPL; rq++) {
        const int q = part * PJ_RPL + rq;  // this range: rows [t0, t1) of each family
        const int t0 = (a.H * q) / PJ_NR, t1 = (a.H * (q + 1)) / PJ_NR;
        float dq[PJ_NB], sq[PJ_NB];
#pragma unroll
        for (int r = 0; r < PJ_NB; r++) dq[r] = sq[r] = 0.f;
        for (int k = 0; k < 3; k++) {
          const float b = a.bound[k];
          const float* Xk = Xs + (size_t)k * a.H * PJ_BLK;
          auto row_update = [&](const float4 x0, const float4 x1, const float4 x2) {
            const float x[PJ_BLK] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w, x2.x, x2.y, x2.z, x2.w};
            float v = 0.f;
#pragma unroll
            for (int c = 0; c < PJ_NB; c++) v = fmaf(x[c], p[c], v);
            const float e_res = fmaxf(v - b, 0.f) - fmaxf(-v - b, 0.f);  // A^T res per row
            const float e_sl = fmaxf(b + v, 0.f) - fmaxf(b - v, 0.f);    // A^T (b - s) per row
#pragma unroll
            for (int c = 0; c < PJ_NB; c++) {
              dq[c] = fmaf(x[c], e_res, dq[c]);
              sq[c] = fmaf(x[c], e_sl, sq[c]);
            }
          };
          int t = t0;
          for (; t + PJ_RG <= t1; t += PJ_RG) {  // a group's LDS loads issue together
            float4 xg[PJ_RG][3];
#pragma unroll
            for (int u = 0; u < PJ_RG; u++)
#pragma unroll
              for (int q3 = 0; q3 < 3; q3++) xg[u][q3] = reinterpret_cast<const float4*>(Xk + (t + u) * PJ_BLK)[q3];
#pragma unroll
            for (int u = 0; u < PJ_RG; u++) row_update(xg[u][0], xg[u][1], xg[u][2]);
          }
          for (; t < t1; t++) {
            const float4* xr = reinterpret_cast<const float4*>(Xk + t * PJ_BLK);
            row_update(xr[0], xr[1], xr[2]);
          }
        }
#pragma unroll
        for (int c = 0; c < PJ_NB; c++) {  // (r0 + r1) within a two-range part; one range: 0 + r0 = r0
          dl[c] += dq[c];
          sl[c] += sq[c];
        }
      }
      // the parts' sums: lanes cl + PJ_CPW q (q = 0..3) swap and add; fp32
      // addition commutes, so all four hold bitwise the same totals
#pragma unroll
      for (int c = 0; c < PJ_NB; c++) {
#pragma unroll
        for (int o = PJ_CPW; o < 64; o <<= 1) {
          dl[c] += __shfl_xor(dl[c], o);
          sl[c] += __shfl_xor(sl[c], o);
        }
      }
#pragma unroll
      for (int r = 0; r < PJ_NB; r++) lam[r] -= a.rho * dl[r];
    }
  }
  // all global stores at the end: nothing before may clobber the tables, so
  // their wave-uniform loads stay scalar (s_load) loads
  if (live && part == 0) {
    if (a.mean && a.xi_samples) {
#pragma unroll
      for (int r = 0; r < PJ_NB; r++) a.xi_samples[(size_t)cand * NV + j * PJ_NB + r] = xi[r];
    }
#pragma unroll
    for (int r = 0; r < PJ_NB; r++) a.xi_out[(size_t)cand * NV + j * PJ_NB + r] = p[r];
  }
}

// ---------------------------------------------------------------------------
// Cholesky of cov + reg I (nv x nv, fp32, right-looking in LDS, one block),
// written transposed and padded for sample_project_kernel: LT[c][r] = L[r][c]
// at padded indices.  A non-PD input yields NaN like jnp.linalg.cholesky.
__global__ void __launch_bounds__(256) cholesky_kernel(const float* __restrict__ cov, int nd, float reg,
                                                        float* __restrict__ LT) {
  __shared__ float A[PJ_MAXD * PJ_NB][PJ_MAXD * PJ_NB + 1];
  __shared__ float Ld[PJ_MAXD * PJ_NB];  // the factor's diagonal (A's diagonal is never overwritten)
  const int nv = nd * PJ_NB, LD = nd * PJ_BLK;
  for (int i = threadIdx.x; i < nv * nv; i += blockDim.x) {
    const int r = i / nv, c = i % nv;
    A[r][c] = cov[i] + (r == c ? reg : 0.f);
  }
  for (int i = threadIdx.x; i < LD * LD; i += blockDim.x) LT[i] = 0.f;
  __syncthreads();
  // right-looking, 16 x 16 threads over the trailing block (no integer
  // division per element: that alone was ~40 instructions an element), two
  // barriers per column
  const int tr = threadIdx.x >> 4, tc = threadIdx.x & 15;
  for (int k = 0; k < nv; k++) {
    const float d = sqrtf(A[k][k]);
    const float id = 1.f / d;
    for (int i = k + 1 + threadIdx.x; i < nv; i += blockDim.x) A[i][k] *= id;
    if (threadIdx.x == 0) Ld[k] = d;
    __syncthreads();
    for (int i = k + 1 + tr; i < nv; i += 16) {
      const float aik = A[i][k];
      for (int c = k + 1 + tc; c <= i; c += 16) A[i][c] -= aik * A[c][k];
    }
    __syncthreads();
  }
  for (int i = threadIdx.x; i < nv * nv; i += blockDim.x) {
    const int r = i / nv, c = i % nv;
    if (c <= r)
      LT[(size_t)((c / PJ_NB) * PJ_BLK + c % PJ_NB) * LD + (r / PJ_NB) * PJ_BLK + r % PJ_NB] = r == c ? Ld[r] : A[r][c];
  }
}

// ---------------------------------------------------------------------------
// top-k: indices of the k smallest costs in stable-argsort order (ascending,
// ties by index, NaN last; -0 == +0).  One 1024-thread block: 4 radix-select
// passes on the order-preserving 32-bit key find the k-th key T, ties at T are
// taken lowest-index first by a block scan in index order, and the k winners
// are bitonic-sorted on (key << 32 | index) in LDS.
__device__ __forceinline__ uint32_t ord_key_nanlast(float c) {
  if (isnan(c)) return 0xFFFFFFFFu;
  const uint32_t u = __float_as_uint(c + 0.0f);  // -0 -> +0
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ void __launch_bounds__(1024) topk_kernel(const float* __restrict__ cost, int stride, int n, int k,
                                                     int* __restrict__ idx_out) {
  __shared__ unsigned long long sel[TOPK_MAX];
  __shared__ uint32_t hist[256];
  __shared__ uint32_t wtot[16];
  __shared__ uint32_t s_prefix, s_krem, s_cnt;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) { s_prefix = 0; s_krem = (uint32_t)k; s_cnt = 0; }
  for (int pass = 0; pass < 4; pass++) {
    const int shift = 24 - 8 * pass;
    for (int i = tid; i < 256; i += 1024) hist[i] = 0;
    __syncthreads();
    const uint32_t prefix = s_prefix;
    for (int i = tid; i < n; i += 1024) {
      const uint32_t key = ord_key_nanlast(cost[(size_t)i * stride]);
      if (pass == 0 || (key >> (shift + 8)) == (prefix >> (shift + 8))) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t cum = 0, krem = s_krem;
      for (int d = 0; d < 256; d++) {
        if (cum + hist[d] >= krem) {
          s_prefix = prefix | ((uint32_t)d << shift);
          s_krem = krem - cum;
          break;
        }
        cum += hist[d];
      }
    }
    __syncthreads();
  }
  const uint32_t T = s_prefix, need = s_krem;  // need >= 1 ties at T are taken
  uint32_t tie_base = 0;
  for (int base = 0; base < n; base += 1024) {
    const int i = base + tid;
    const uint32_t key = i < n ? ord_key_nanlast(cost[(size_t)i * stride]) : 0u;
    const bool eq = i < n && key == T;
    const unsigned long long bal = __ballot(eq);
    const uint32_t before = (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wtot[wid] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t off = tie_base, tot = 0;
    for (int w = 0; w < 16; w++) {
      if (w < wid) off += wtot[w];
      tot += wtot[w];
    }
    const bool take = i < n && (key < T || (eq && off + before < need));
    if (take) {
      const uint32_t pos = atomicAdd(&s_cnt, 1u);
      sel[pos] = ((unsigned long long)key << 32) | (uint32_t)i;
    }
    tie_base += tot;
    __syncthreads();
  }
  int K2 = 1;
  while (K2 < k) K2 <<= 1;
  for (int i = k + tid; i < K2; i += 1024) sel[i] = ~0ull;
  __syncthreads();
  for (int size = 2; size <= K2; size <<= 1) {
    for (int stride2 = size >> 1; stride2 > 0; stride2 >>= 1) {
      for (int i = tid; i < K2; i += 1024) {
        const int partner = i ^ stride2;
        if (partner > i) {
          const bool up = (i & size) == 0;
          const unsigned long long x = sel[i], y = sel[partner];
          if ((x > y) == up) { sel[i] = y; sel[partner] = x; }
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < k; i += 1024) idx_out[i] = (int)(uint32_t)(sel[i] & 0xFFFFFFFFull);
}

// ---------------------------------------------------------------------------
// weighted mean / covariance of the elites (compute_mean_cov, :325-335), one
// 1024-thread block; mean and cov are updated in place.
constexpr int CU_CHUNK = 64;

__global__ void __launch_bounds__(1024) cem_update_kernel(const float* __restrict__ xi, int nv,
                                                           const float* __restrict__ cost, int stride,
                                                           const int* __restrict__ idx, int k, float lamda,
                                                           float alpha_mean, float alpha_cov, float reg,
                                                           float* mean, float* cov) {
  __shared__ float w[TOPK_MAX];
  __shared__ float d[CU_CHUNK][PJ_MAXD * PJ_NB + 1];
  __shared__ float red[1024 / 64];
  __shared__ float msum[16][PJ_MAXD * PJ_NB];
  __shared__ float mnew[PJ_MAXD * PJ_NB];
  __shared__ float s_cmin, s_sw;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // c_min = jnp.min(cost_ellite): NaN propagates
  float cm = INFINITY;
  bool nan = false;
  for (int e = tid; e < k; e += 1024) {
    const float c = cost[(size_t)idx[e] * stride];
    nan |= isnan(c);
    cm = fminf(cm, c);
  }
  nan = __any(nan);
  for (int o = 32; o > 0; o >>= 1) cm = fminf(cm, __shfl_xor(cm, o));
  if (lane == 0) red[wid] = nan ? NAN : cm;
  __syncthreads();
  if (tid == 0) {
    float m = INFINITY;
    bool anynan = false;
    for (int i = 0; i < 16; i++) { anynan |= isnan(red[i]); m = fminf(m, red[i]); }
    s_cmin = anynan ? NAN : m;
  }
  __syncthreads();
  const float cmin = s_cmin;
  float sw = 0.f;
  for (int e = tid; e < k; e += 1024) {
    const float we = expf(-(1.0f / lamda) * (cost[(size_t)idx[e] * stride] - cmin));
    w[e] = we;
    sw += we;
  }
  for (int o = 32; o > 0; o >>= 1) sw += __shfl_xor(sw, o);
  __syncthreads();
  if (lane == 0) red[wid] = sw;
  __syncthreads();
  if (tid == 0) {
    float s = 0.f;
    for (int i = 0; i < 16; i++) s += red[i];
    s_sw = s;
  }
  __syncthreads();
  const float swt = s_sw;
  // mean: thread (g, c), g < 15 groups of elites
  const int G = 1024 / nv;
  {
    const int g = tid / nv, c = tid % nv;
    float acc = 0.f;
    if (g < G)
      for (int e = g; e < k; e += G) acc = fmaf(xi[(size_t)idx[e] * nv + c], w[e], acc);
    if (g < G) msum[g][c] = acc;
  }
  __syncthreads();
  if (tid < nv) {
    float s = 0.f;
    for (int g = 0; g < G; g++) s += msum[g][tid];
    mnew[tid] = (1.f - alpha_mean) * mean[tid] + alpha_mean * (s / swt);
  }
  __syncthreads();
  // cov: thread owns entries tid, tid+1024, ... of the nv x nv matrix
  constexpr int MAXE = (PJ_MAXD * PJ_NB * PJ_MAXD * PJ_NB + 1023) / 1024;
  float acc[MAXE];
#pragma unroll
  for (int q = 0; q < MAXE; q++) acc[q] = 0.f;
  for (int e0 = 0; e0 < k; e0 += CU_CHUNK) {
    const int ne = min(CU_CHUNK, k - e0);
    for (int i = tid; i < ne * nv; i += 1024) {
      const int e = i / nv, c = i % nv;
      d[e][c] = xi[(size_t)idx[e0 + e] * nv + c] - mnew[c];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < MAXE; q++) {
      const int ent = tid + q * 1024;
      if (ent < nv * nv) {
        const int r = ent / nv, c = ent % nv;
        float s = acc[q];
        for (int e = 0; e < ne; e++) s = fmaf(d[e][r] * d[e][c], w[e0 + e], s);  // outer(d, d) * w: symmetric
        acc[q] = s;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < MAXE; q++) {
    const int ent = tid + q * 1024;
    if (ent < nv * nv) {
      const int r = ent / nv, c = ent % nv;
      cov[ent] = (1.f - alpha_cov) * cov[ent] + alpha_cov * (acc[q] / swt) + (r == c ? reg : 0.f);
    }
  }
  if (tid < nv) mean[tid] = mnew[tid];
}

}  // namespace mpcr
