// rollout.hip — fused basis -> H MuJoCo-semantics steps -> cost kernel for
// gfx950 (CDNA4).  One 64-lane wavefront (one workgroup) owns one candidate
// rollout for the whole horizon; per step the lanes run in parallel over
// bodies (kinematics by pointer jumping along the chain), dofs (cdof, RNE,
// passive), (dof, dof) entries (CRB mass matrix), collision pairs (narrow
// phase), (contact, dof) entries (contact Jacobians) and constraint rows
// (impedance, Newton line search).  The two dense SPD solves per step
// (M and the Newton Hessian) are done row-per-lane in registers with DPP
// row broadcasts (nv <= 16) or v_readlane (the 32-wide dual-arm variant): no
// LDS round trips inside the factorisation.  Built as its own translation
// unit (flags: manipulator_mujoco_amd/build.py); host side in engine.hip.
//
// Semantics restated (same definitions as oracle/mpcr_oracle.c):
//   rollout / output timing  SBP/mjx_planner.py:251-274
//   cost                     SBP/mjx_planner.py:276-303
//   mjx.step                 mujoco-mjx 3.3.1 (third party)
#include <cstdlib>
#include <atomic>

#include "rollout.h"
#include "../../include/mpcr_model.h"  // MPCR_LUT_R (the engine's hull start table)

namespace mpcr {

// ---------------------------------------------------------------------------
// diagnostic phase stamps (separate -DMPCR_PROFILE build; never in the timed one)
#ifdef MPCR_PROFILE
#define PROF_DECL unsigned long long prof_acc[32] = {0}; unsigned long long prof_last = __builtin_amdgcn_s_memtime();
#define STAMP(i)                                              \
  do {                                                        \
    unsigned long long now_ = __builtin_amdgcn_s_memtime();   \
    prof_acc[i] += now_ - prof_last;                          \
    prof_last = now_;                                         \
  } while (0)
// (a candidate's second wave, WPC = 2, into slots 32..63: per-wave critical paths)
#define PROF_FLUSH                                                          \
  if (lane == 0 && args.prof)                                               \
    for (int i_ = 0; i_ < 32; i_++) atomicAdd(&args.prof[i_ + 32 * (threadIdx.x >> 6)], prof_acc[i_]);
// wave-level event counter (first active lane adds 1; -DMPCR_PROFILE_COUNTS
// only: the shared atomics distort the cycle shares)
#ifdef MPCR_PROFILE_COUNTS
#define PROF_COUNT(m, i)                                                                  \
  do {                                                                                    \
    if ((m)->prof && (int)__lane_id() == __builtin_ctzll(__ballot(1))) atomicAdd((m)->prof + (i), 1ull); \
  } while (0)
#else
#define PROF_COUNT(m, i)
#endif
// sub-phase stamps inside a device function (one atomic per stamp and wave)
#define PSTAMP_DECL unsigned long long pst_ = __builtin_amdgcn_s_memtime();
#define PSTAMP(m, i)                                                                       \
  do {                                                                                     \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();                          \
    if ((m)->prof && (int)__lane_id() == 0) atomicAdd((m)->prof + (i) + 32 * (threadIdx.x >> 6), now_ - pst_); \
    pst_ = now_;                                                                           \
  } while (0)
#else
#define PSTAMP_DECL
#define PSTAMP(m, i)
#define PROF_DECL
#define STAMP(i)
#define PROF_FLUSH
#define PROF_COUNT(m, i)
#endif
// Pacing (load balance of a one-round launch): at N = 4096 every candidate is
// resident at once (4 waves per SIMD) and the launch ends with the slowest
// candidate, ~18 % after the mean one (tools/wavetime.py).  Each wave posts
// the step it is on in its SIMD's slot group and takes an issue priority
// equal to the number of its SIMD mates ahead of it, so the waves sharing a
// SIMD progress together and the SIMD drains when its total work is done.
#ifndef MPCR_PACE
#define MPCR_PACE 1
#endif
// pacing in the dual-arm kernel too: 1.7 % slower at 7 blocks per CU (2.3
// backfilled rounds), ~0.8 % faster at 8 (C4 4096 x 100: 33.6-34.0 vs
// 34.1 ms; 8192 x 50: 30.35-30.45 vs 30.57-30.79 ms)
#ifndef MPCR_W_PACE
#define MPCR_W_PACE 1
#endif
// a mate counts as ahead when it is more than MPCR_PACE_LAG steps ahead
#ifndef MPCR_PACE_LAG
#define MPCR_PACE_LAG 0
#endif
// where the mates' progress read at the step start is consumed: 0 before the
// collision phase (mid-step), 1 at the next step's start, 2 before Newton
#ifndef MPCR_PACE_AT
#define MPCR_PACE_AT 0
#endif
#define PACE_SETPRIO() \
  if (pace) {  /* priority = SIMD mates ahead of this wave (0..3) */ \
  const int ahead = __popcll(__ballot(lane < 16 && lane != pace_own && pace_v != ~0u && pace_v > (unsigned)t + MPCR_PACE_LAG)); \
  if (ahead >= 3) __builtin_amdgcn_s_setprio(3); \
  else if (ahead == 2) __builtin_amdgcn_s_setprio(2); \
  else if (ahead == 1) __builtin_amdgcn_s_setprio(1); \
  else __builtin_amdgcn_s_setprio(0); \
  }

// ablation builds (timing attribution only; results are wrong): skip the
// capsule-box deepest-point search / the narrow-phase functions in the mask
#ifndef MPCR_ABL_DEEP
#define MPCR_ABL_DEEP 0
#endif
#ifndef MPCR_CB_SKIP
#define MPCR_CB_SKIP 1  // capsule-box: skip the interior knots when no lane's minimum is inside (narrow_lane)
#endif
#ifndef MPCR_ABL_FUNC
#define MPCR_ABL_FUNC 0
#endif
#ifndef MPCR_WPC2_MAX_N_DEFAULT
#define MPCR_WPC2_MAX_N_DEFAULT 2048  // batches up to this size run two waves per candidate (narrow variant;
                                      // C3 512 / 1024 / 2048: 1.38 / 1.43 / 1.52 -> 1.07 / 1.09 / 1.20 ms,
                                      // 4096: 1.77 -> 3.03 ms, the one-wave kernel stays)
#endif
// wide Newton's J^T f / J^T D J on two MFMA accumulators with batched row loads
#ifndef MPCR_W_MFMA_SPLIT
#define MPCR_W_MFMA_SPLIT 0  // measured: C4 50.97 vs 50.90 ms (noise), results move by an ulp: not kept
#endif
#ifndef MPCR_TD_TABLE
#define MPCR_TD_TABLE 1
#endif
// instruction-count attribution builds (-DMPCR_STOP_AFTER=k, diagnostic only):
// the step ends right after phase stamp k, so PMC differences between k and
// the previous stop are that phase's instructions
#ifdef MPCR_STOP_AFTER
#define STOP_AT(k) \
  if (MPCR_STOP_AFTER == (k)) continue;
#else
#define STOP_AT(k)
#endif

// ---------------------------------------------------------------------------
// wave helpers

// Address spaces at the entry of a non-inlined device function: its pointer
// arguments are generic, so without these the model reads, the LDS image and
// the caller's contact arrays all go through flat instructions (which also
// count against the LDS wait counter)
// (device pass only: the host pass parses device bodies with other builtin signatures)
#if defined(__HIP_DEVICE_COMPILE__)
#define ASSUME_GLOBAL(p) __builtin_assume(!__builtin_amdgcn_is_shared((const void*)(p)) && \
                                          !__builtin_amdgcn_is_private((const void*)(p)))
#define ASSUME_LDS(p) __builtin_assume(__builtin_amdgcn_is_shared((const void*)(p)))
#define ASSUME_PRIVATE(p) __builtin_assume(__builtin_amdgcn_is_private((const void*)(p)))
#else
#define ASSUME_GLOBAL(p)
#define ASSUME_LDS(p)
#define ASSUME_PRIVATE(p)
#endif
// the model pointer as a wave-uniform (SGPR) global pointer: a non-inlined
// function receives it in VGPRs, and its field reads then become per-lane
// vector loads instead of scalar ones
__device__ __forceinline__ const MPCR_GMEM DevModel* uniform_model(const DevModel* p) {
  const unsigned long long a = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a), hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  return reinterpret_cast<const MPCR_GMEM DevModel*>(((unsigned long long)hi << 32) | lo);
}

__device__ __forceinline__ float rdlane(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// full-wave sum, result uniform: DPP inside each 16-lane row (quad_perm
// [1,0,3,2], [2,3,0,1], row_ror:4, row_ror:8), then the GCN row_bcast:15 /
// row_bcast:31 steps carry the row sums into lane 63, one readlane.  No LDS
// traffic (a __shfl_xor butterfly is 6 dependent ds_bpermute round trips).
template <int CTRL, int ROWS>
__device__ __forceinline__ float dppf_rows(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROWS, 0xF, false));
}
__device__ __forceinline__ float wsum(float v) {
  v += dppf<0xB1>(v);
  v += dppf<0x4E>(v);
  v += dppf<0x124>(v);
  v += dppf<0x128>(v);
  v += dppf_rows<0x142, 0xA>(v);  // row_bcast:15 into rows 1, 3
  v += dppf_rows<0x143, 0xC>(v);  // row_bcast:31 into rows 2, 3
  return rdlane(v, 63);
}
__device__ __forceinline__ int lanes_below(unsigned long long mask) {
  return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
}
// exclusive prefix sum of small per-lane counts (0 .. 2^BITS - 1) by bit-plane ballots
template <int BITS = 3>
__device__ __forceinline__ int wscan_excl(int v, int& total) {
  int pre = 0, tot = 0;
#pragma unroll
  for (int bit = 0; bit < BITS; bit++) {
    const unsigned long long mk = __ballot((v >> bit) & 1);
    pre += lanes_below(mk) << bit;
    tot += __popcll(mk) << bit;
  }
  total = tot;
  return pre;
}
// Phase barrier of one candidate's wave: orders its lanes' LDS / global
// accesses (the workgroup-scope fences of __syncthreads, without s_barrier).
// A one-wave workgroup measured the same with either (1.963 vs 1.964 ms on C3);
// the two-wave variant (WPC = 2) needs the wave-local form, its waves meet at
// block_sync() only.
__device__ __forceinline__ void sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
__device__ __forceinline__ void block_sync() { __syncthreads(); }

// Candidate groups: a wave may carry CPW candidates of HL = 64 / CPW lanes
// (lanes [32 h, 32 h + 32) for candidate h when CPW = 2).  These are the
// group-local forms of the wave primitives above; ballots keep their bits in
// place, restricted to the own group, so lanes_below / __popcll apply as is.
template <int CPW>
__device__ __forceinline__ int hlane() { return threadIdx.x & (WAVE / CPW - 1); }
template <int CPW>
__device__ __forceinline__ int hbase() { return threadIdx.x & (WAVE - WAVE / CPW); }
template <int CPW>
__device__ __forceinline__ unsigned long long hmask() {
  if constexpr (CPW == 1) return ~0ull;
  else return threadIdx.x >= 32 ? 0xffffffff00000000ull : 0xffffffffull;
}
template <int CPW>
__device__ __forceinline__ unsigned long long hballot(bool p) { return __ballot(p) & hmask<CPW>(); }
template <int CPW>
__device__ __forceinline__ float hrdlane(float v, int l) {
  if constexpr (CPW == 1) return rdlane(v, l);
  else return threadIdx.x >= 32 ? rdlane(v, 32 + l) : rdlane(v, l);
}
template <int CPW>
__device__ __forceinline__ float hsum(float v) {
  if constexpr (CPW == 1) {
    return wsum(v);
  } else {
    v += dppf<0xB1>(v);
    v += dppf<0x4E>(v);
    v += dppf<0x124>(v);
    v += dppf<0x128>(v);
    v += dppf_rows<0x142, 0xA>(v);  // rows 1, 3 += rows 0, 2: group sums in lanes 31, 63
    return threadIdx.x >= 32 ? rdlane(v, 63) : rdlane(v, 31);
  }
}
template <int CPW, class T>
__device__ __forceinline__ T hshfl(T x, int src) { return __shfl(x, src + hbase<CPW>()); }
template <int CPW>
__device__ __forceinline__ int hscan_excl(int v, int& total) {
  int pre = 0, tot = 0;
#pragma unroll
  for (int bit = 0; bit < 3; bit++) {
    const unsigned long long mk = hballot<CPW>((v >> bit) & 1);
    pre += lanes_below(mk) << bit;
    tot += __popcll(mk) << bit;
  }
  total = tot;
  return pre;
}

// ---------------------------------------------------------------------------
// small vector math

__device__ __forceinline__ void qmul(float r[4], const float a[4], const float b[4]) {
  float t0 = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  float t1 = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  float t2 = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  float t3 = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3;
}
__device__ __forceinline__ void q2m(float m[9], const float q[4]) {
  float w = q[0], x = q[1], y = q[2], z = q[3];
  m[0] = 1 - 2 * (y * y + z * z); m[1] = 2 * (x * y - w * z); m[2] = 2 * (x * z + w * y);
  m[3] = 2 * (x * y + w * z); m[4] = 1 - 2 * (x * x + z * z); m[5] = 2 * (y * z - w * x);
  m[6] = 2 * (x * z - w * y); m[7] = 2 * (y * z + w * x); m[8] = 1 - 2 * (x * x + y * y);
}
__device__ __forceinline__ void mv(float r[3], const float m[9], const float v[3]) {
  float a = m[0] * v[0] + m[1] * v[1] + m[2] * v[2];
  float b = m[3] * v[0] + m[4] * v[1] + m[5] * v[2];
  float c = m[6] * v[0] + m[7] * v[1] + m[8] * v[2];
  r[0] = a; r[1] = b; r[2] = c;
}
__device__ __forceinline__ void mtv(float r[3], const float m[9], const float v[3]) {
  float a = m[0] * v[0] + m[3] * v[1] + m[6] * v[2];
  float b = m[1] * v[0] + m[4] * v[1] + m[7] * v[2];
  float c = m[2] * v[0] + m[5] * v[1] + m[8] * v[2];
  r[0] = a; r[1] = b; r[2] = c;
}
__device__ __forceinline__ void cross(float r[3], const float a[3], const float b[3]) {
  float x = a[1] * b[2] - a[2] * b[1];
  float y = a[2] * b[0] - a[0] * b[2];
  float z = a[0] * b[1] - a[1] * b[0];
  r[0] = x; r[1] = y; r[2] = z;
}
__device__ __forceinline__ float dot3(const float a[3], const float b[3]) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
__device__ __forceinline__ float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
// N-wide dot product of an LDS row (16-byte aligned) with an LDS vector
template <int N>
__device__ __forceinline__ float dotN(const float* row, const float* vec) {
  const float4* r = reinterpret_cast<const float4*>(row);
  const float4* v = reinterpret_cast<const float4*>(vec);
  float acc = 0.f;
#pragma unroll
  for (int q = 0; q < N / 4; q++) {
    const float4 a = r[q], x = v[q];
    acc = fmaf(a.x, x.x, acc); acc = fmaf(a.y, x.y, acc); acc = fmaf(a.z, x.z, acc); acc = fmaf(a.w, x.w, acc);
  }
  return acc;
}

// spatial algebra (MuJoCo layout, see oracle/mpcr_oracle.c)
__device__ __forceinline__ void mul_inert_vec(float r[6], const float* i, const float* v) {
  r[0] = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
  r[1] = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
  r[2] = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
  r[3] = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
  r[4] = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
  r[5] = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
}
__device__ __forceinline__ void cross_motion(float r[6], const float v[6], const float u[6]) {
  float a[3], b[3], c[3];
  cross(a, v, u);
  cross(b, v, u + 3);
  cross(c, v + 3, u);
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2];
  r[3] = b[0] + c[0]; r[4] = b[1] + c[1]; r[5] = b[2] + c[2];
}
__device__ __forceinline__ void cross_force(float r[6], const float v[6], const float f[6]) {
  float a[3], b[3], c[3];
  cross(a, v, f);
  cross(b, v + 3, f + 3);
  cross(c, v, f + 3);
  r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2];
  r[3] = c[0]; r[4] = c[1]; r[5] = c[2];
}

// ---------------------------------------------------------------------------
// dense SPD solve, row-per-lane in registers.  Lane i (< DX_NV) holds row i
// of A in a[]; rows >= n must be identity rows.  On return a[] holds row i of
// the lower Cholesky factor.  x = A^-1 b for b held one value per lane.

// All DX_NV pivots run even when nv is smaller: a run-time exit inside the
// unrolled chain breaks it into blocks the scheduler cannot overlap
// (measured 4.07 -> 4.94 ms), while the padded pivots cost 2/16 of it.
template <int N>
__device__ __forceinline__ void chol_rows(float (&a)[N], int lane) {
#pragma unroll
  for (int k = 0; k < N; k++) {
    float dkk = sqrtf(fmaxf(rdlane(a[k], k), kMinVal));
    float lik = lane == k ? dkk : (lane > k ? a[k] / dkk : 0.f);
    a[k] = lik;
#pragma unroll
    for (int j = k + 1; j < N; j++) {
      float ljk = rdlane(lik, j);
      a[j] = fmaf(-lik, ljk, a[j]);
    }
  }
}

// x = L^-T L^-1 b with lane i holding row i of L in l[].  Forward pass: lane
// k finalises y_k, one v_readlane broadcasts it, every lane updates its own
// accumulator with its own register l[k].  For the backward pass each lane
// needs its COLUMN of L: the rows are scattered transposed to the LDS scratch
// Lt[DX_NV][LDL] once, each lane reads its column back with 4 ds_read_b128,
// and the same broadcast chain runs backwards.  32 readlanes per solve.
// Returns x[lane].  Must be called by all lanes (one barrier).
template <int N, int LDL>
__device__ __forceinline__ float chol_solve(const float (&l)[N], float b, int lane, float* Lt) {
  if (lane < N) {
#pragma unroll
    for (int j = 0; j < N; j++) Lt[j * LDL + lane] = l[j];
  }
  float acc = b, y = 0.f;
#pragma unroll
  for (int k = 0; k < N; k++) {
    const float yk = rdlane(acc, k) / rdlane(l[k], k);
    if (lane > k) acc = fmaf(-l[k], yk, acc);
    if (lane == k) y = yk;
  }
  sync();
  float lt[N];
  {
    const float4* col = reinterpret_cast<const float4*>(Lt + (lane < N ? lane : 0) * LDL);
#pragma unroll
    for (int q = 0; q < N / 4; q++) {
      const float4 v = col[q];
      lt[4 * q] = v.x; lt[4 * q + 1] = v.y; lt[4 * q + 2] = v.z; lt[4 * q + 3] = v.w;
    }
  }
  float x = 0.f;
  acc = y;
#pragma unroll
  for (int k = N - 1; k >= 0; k--) {
    const float xk = rdlane(acc, k) / rdlane(l[k], k);
    if (lane < k) acc = fmaf(-lt[k], xk, acc);
    if (lane == k) x = xk;
  }
  sync();
  return x;
}

// The same factorisation and solve for N = 16 (narrow variant) with DPP row
// broadcasts instead of v_readlane: row_newbcast:j hands lane j's value to
// every lane of its 16-lane row, and as the src0 modifier of v_fmac_f32 it
// makes each (k, j) update of the right-looking factorisation ONE VALU
// instruction (readlane + fma before, plus the SGPR hazards).  Lanes 16..63
// run the same code on their own rows and their results are ignored.
template <int J>
__device__ __forceinline__ float rbc(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x150 + J, 0xF, 0xF, true));
}
// acc -= bcast_J(src) * own.  NOP: src was just written by a VALU op (DPP
// reads need 2 wait states; the compiler does not track them in inline asm)
template <int J, bool NOP>
__device__ __forceinline__ void fnmac_bc(float& acc, float src, float own) {
  if constexpr (NOP)
    asm("s_nop 1\n\tv_fmac_f32_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
        : "+v"(acc) : "v"(src), "v"(own), "n"(J));
  else
    asm("v_fmac_f32_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
        : "+v"(acc) : "v"(src), "v"(own), "n"(J));
}
template <int K, int J>
struct Chol16Upd {  // a[j] -= l[j][k] * l[i][k] for j = J..15
  static __device__ __forceinline__ void run(float (&a)[16], float lik) {
    fnmac_bc<J, J == K + 1>(a[J], lik, lik);
    Chol16Upd<K, J + 1>::run(a, lik);
  }
};
template <int K>
struct Chol16Upd<K, 16> {
  static __device__ __forceinline__ void run(float (&)[16], float) {}
};
// The factor is kept with a ZERO diagonal: l[i][i] lives only as its inverse
// in dinv (lane i).  The sweeps then leave lane K's accumulator alone when
// they broadcast its value, and read every result off at the end (acc * dinv)
// instead of capturing it with a per-step select.
template <int K>
struct Chol16 {  // column K; dinv collects 1 / l[i][i] at lane i
  static __device__ __forceinline__ void run(float (&a)[16], float& dinv, int lane) {
    const float dkk = sqrtf(fmaxf(rbc<K>(a[K]), kMinVal));
    const float inv = 1.f / dkk;
    const float lik = lane > K ? a[K] * inv : 0.f;
    a[K] = lik;
    dinv = lane == K ? inv : dinv;
    Chol16Upd<K, K + 1>::run(a, lik);
    Chol16<K + 1>::run(a, dinv, lane);
  }
};
template <>
struct Chol16<16> {
  static __device__ __forceinline__ void run(float (&)[16], float&, int) {}
};
// forward (L y = b) / backward (L^T x = y) sweeps: lane K's value is final
// at step K, t = acc / l_KK, and one fused DPP FMA hands it to the other
// lanes' updates (lanes already final and lane K see zero coefficients: l is
// triangular with a zero diagonal); the results are acc * dinv afterwards
template <int K, int STEP>
struct Sweep16 {
  static __device__ __forceinline__ void run(const float (&c)[16], float& acc, float dinv) {
    const float t = acc * dinv;
    fnmac_bc<K, true>(acc, t, c[K]);
    Sweep16<K + STEP, STEP>::run(c, acc, dinv);
  }
};
template <int STEP>
struct Sweep16<16, STEP> {
  static __device__ __forceinline__ void run(const float (&)[16], float&, float) {}
};
template <int STEP>
struct Sweep16<-1, STEP> {
  static __device__ __forceinline__ void run(const float (&)[16], float&, float) {}
};
// the blocked (per-tree) Cholesky for M and uncoupled Newton Hessians
#ifndef MPCR_BLOCK_CHOL
#define MPCR_BLOCK_CHOL 1
#endif
// MPCR_CHOL_LANE_LAUNDER: re-derive the lane compares inside the solves (one
// v_cmp each) instead of letting them be hoisted into spilled SGPR pairs
#ifndef MPCR_CHOL_LANE_LAUNDER
#define MPCR_CHOL_LANE_LAUNDER 1
#endif
__device__ __forceinline__ void chol16(float (&a)[16], float& dinv, int lane) {
  if (MPCR_CHOL_LANE_LAUNDER) asm volatile("" : "+v"(lane));
  dinv = 0.f;
  Chol16<0>::run(a, dinv, lane);
}
// Blocked variant for block-diagonal systems (the mass matrix is block
// diagonal by kinematic tree): tree t's <= 8 dofs are rows of lanes 16 t ..
// 16 t + 7, and row_newbcast:K broadcasts each tree's K-th row to its own
// lanes, so all trees factor in ONE 8-column chain (36 fused updates instead
// of 120) -- the same operations per block as the dense factorisation
// (off-block entries are exact zeros there), in the same order.
template <int N, int K, int J>
struct CholNUpd {
  static __device__ __forceinline__ void run(float (&a)[N], float lik) {
    fnmac_bc<J, J == K + 1>(a[J], lik, lik);
    CholNUpd<N, K, J + 1>::run(a, lik);
  }
};
template <int N, int K>
struct CholNUpd<N, K, N> {
  static __device__ __forceinline__ void run(float (&)[N], float) {}
};
template <int N, int K>
struct CholN {  // lr: the lane's row within its 16-lane DPP row
  static __device__ __forceinline__ void run(float (&a)[N], float& dinv, int lr) {
    const float dkk = sqrtf(fmaxf(rbc<K>(a[K]), kMinVal));
    const float inv = 1.f / dkk;
    const float lik = lr > K ? a[K] * inv : 0.f;
    a[K] = lik;
    dinv = lr == K ? inv : dinv;
    CholNUpd<N, K, K + 1>::run(a, lik);
    CholN<N, K + 1>::run(a, dinv, lr);
  }
};
template <int N>
struct CholN<N, N> {
  static __device__ __forceinline__ void run(float (&)[N], float&, int) {}
};
template <int N, int K, int STEP>
struct SweepN {
  static __device__ __forceinline__ void run(const float (&c)[N], float& acc, float dinv) {
    const float t = acc * dinv;
    fnmac_bc<K, true>(acc, t, c[K]);
    SweepN<N, K + STEP, STEP>::run(c, acc, dinv);
  }
};
template <int N, int STEP>
struct SweepN<N, N, STEP> {
  static __device__ __forceinline__ void run(const float (&)[N], float&, float) {}
};
template <int N, int STEP>
struct SweepN<N, -1, STEP> {
  static __device__ __forceinline__ void run(const float (&)[N], float&, float) {}
};
// x = A^-1 b for a symmetric A that is block diagonal by kinematic tree (tree
// t's <= N dofs on lanes 16 t ..), elem(d, dj) = A[d][dj]; b and x are
// dof-indexed LDS vectors (x may alias b).  Lt: 4 N^2-float LDS scratch (it
// may alias A's storage: every element is read before the first write).  Must
// be called by all lanes (two barriers).
// (split in two for a factor computed ahead of its solve, possibly on
// another wave: blocked_factor, then blocked_sweep -- the same operations)
template <int N, class F>
__device__ __forceinline__ void blocked_factor(const DevModel* __restrict__ m, F&& elem, int lane, float (&a)[N],
                                               float& dinv) {
  static_assert(N == 8 || N == 16, "blocked Cholesky width");
  if (MPCR_CHOL_LANE_LAUNDER) asm volatile("" : "+v"(lane));
  const int lr = lane & 15, lb = lane & ~15;
  const int d = m->blane_dof[lane];
#pragma unroll
  for (int j = 0; j < N; j++) {
    const int dj = m->blane_dof[lb + j];
    a[j] = (d >= 0 && dj >= 0) ? elem(d, dj) : (j == lr ? 1.f : 0.f);
  }
  dinv = 0.f;
  CholN<N, 0>::run(a, dinv, lr);
}
template <int N>
__device__ __forceinline__ void blocked_sweep(const DevModel* __restrict__ m, const float (&a)[N], float dinv,
                                              const float* bv, float* xv, int lane, float* Lt) {
  if (MPCR_CHOL_LANE_LAUNDER) asm volatile("" : "+v"(lane));
  const int lr = lane & 15, t = lane >> 4;
  const int d = m->blane_dof[lane];
  float acc = d >= 0 ? bv[d] : 0.f;
  SweepN<N, 0, 1>::run(a, acc, dinv);
  const float y = acc * dinv;
  if (lr < N) {
#pragma unroll
    for (int j = 0; j < N; j++) Lt[t * N * N + j * N + lr] = a[j];
  }
  sync();
  float lt[N];
  {
    const float4* col = reinterpret_cast<const float4*>(Lt + t * N * N + (lr & (N - 1)) * N);
#pragma unroll
    for (int q = 0; q < N / 4; q++) {
      const float4 v = col[q];
      lt[4 * q] = v.x; lt[4 * q + 1] = v.y; lt[4 * q + 2] = v.z; lt[4 * q + 3] = v.w;
    }
  }
  acc = y;
  SweepN<N, N - 1, -1>::run(lt, acc, dinv);
  const float x = acc * dinv;
  sync();
  if (d >= 0) xv[d] = x;
}
template <int N, class F>
__device__ __forceinline__ void blocked_solve(const DevModel* __restrict__ m, F&& elem, const float* bv, float* xv,
                                              int lane, float* Lt) {
  float a[N], dinv;
  blocked_factor<N>(m, elem, lane, a, dinv);
  blocked_sweep<N>(m, a, dinv, bv, xv, lane, Lt);
}
// the blocked path for a kernel variant of NVW dofs: 8-wide chains in the
// narrow kernel (trees <= 8 dofs), 16-wide in the dual-arm one (trees <= 16)
template <int NVW>
__device__ __forceinline__ bool blk_usable(const DevModel* __restrict__ m) {
  return MPCR_BLOCK_CHOL && (NVW == 16 ? m->blk_n == 8 : m->blk_n != 0);
}
template <int NVW, class F>
__device__ __forceinline__ void blk_solve(const DevModel* __restrict__ m, F&& elem, const float* bv, float* xv,
                                          int lane, float* Lt) {
  blocked_solve<NVW == 16 ? 8 : 16>(m, elem, bv, xv, lane, Lt);
}

// x = L^-T L^-1 b (lane i: row i of L in l[]); Lt: LDS transpose scratch
template <int LDL>
__device__ __forceinline__ float chol16_solve(const float (&l)[16], float dinv, float b, int lane, float* Lt) {
  if (MPCR_CHOL_LANE_LAUNDER) asm volatile("" : "+v"(lane));
  if (lane < 16) {
#pragma unroll
    for (int j = 0; j < 16; j++) Lt[j * LDL + lane] = l[j];
  }
  float acc = b;
  Sweep16<0, 1>::run(l, acc, dinv);
  const float y = acc * dinv;
  sync();
  float lt[16];
  {
    const float4* col = reinterpret_cast<const float4*>(Lt + (lane & 15) * LDL);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const float4 v = col[q];
      lt[4 * q] = v.x; lt[4 * q + 1] = v.y; lt[4 * q + 2] = v.z; lt[4 * q + 3] = v.w;
    }
  }
  acc = y;
  Sweep16<15, -1>::run(lt, acc, dinv);
  const float x = acc * dinv;
  sync();
  return x;
}

// ---------------------------------------------------------------------------
// narrow phase (contact definitions identical to the oracle's)

__device__ __forceinline__ void seg_seg(const float p1[3], const float d1[3], const float p2[3], const float d2[3],
                                        float* sc, float* tc) {
  float r[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]};
  float a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
  float s, t;
  if (a <= kMinVal && e <= kMinVal) { *sc = 0; *tc = 0; return; }
  if (a <= kMinVal) {
    s = 0; t = clampf(f / e, 0, 1);
  } else {
    float c = dot3(d1, r);
    if (e <= kMinVal) {
      t = 0; s = clampf(-c / a, 0, 1);
    } else {
      float b = dot3(d1, d2), den = a * e - b * b;
      s = den > 1e-12f * a * e ? clampf((b * f - c * e) / den, 0, 1) : 0.f;
      t = (b * s + f) / e;
      if (t < 0) { t = 0; s = clampf(-c / a, 0, 1); }
      else if (t > 1) { t = 1; s = clampf((b - c) / a, 0, 1); }
    }
  }
  *sc = s; *tc = t;
}

__device__ __forceinline__ float point_box(const float p[3], const float h[3], float nl[3], float q[3]) {
  float out2 = 0, o[3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    q[k] = clampf(p[k], -h[k], h[k]);
    o[k] = q[k] - p[k];
    out2 += o[k] * o[k];
  }
  if (out2 > 0) {
    const float l = sqrtf(out2);
#pragma unroll
    for (int k = 0; k < 3; k++) nl[k] = o[k] / l;
    return l;
  }
  // inside: the deepest face is argmax_k |p_k| - h_k; ties within 1 um go to
  // the lower axis and a point on the box's mid-plane to the + face (the
  // oracle's point_box rule)
  const float g0 = fabsf(p[0]) - h[0], g1 = fabsf(p[1]) - h[1], g2 = fabsf(p[2]) - h[2];
  int best = 0;
  float g = g0;
  if (g1 > g + 1e-6f) { g = g1; best = 1; }
  if (g2 > g + 1e-6f) { g = g2; best = 2; }
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const float sg = p[k] >= -1e-6f ? 1.f : -1.f;
    nl[k] = k == best ? -sg : 0.f;
    q[k] = k == best ? sg * h[k] : p[k];
  }
  return g;
}

// ---------------------------------------------------------------------------
// general convex narrow phase (dual-arm class only): support functions of
// sphere / capsule / cylinder / box / mesh convex hull and Minkowski portal
// refinement, the same algorithm and tolerances as the oracle's mpr()
// (libccd MPR; one penetration contact per pair)

#ifndef MPCR_MPR_TOL
#define MPCR_MPR_TOL 1e-6f  // MuJoCo's ccd_tolerance (round 3; 1e-5 before)
#endif
#ifndef MPCR_MPR_ITER
#define MPCR_MPR_ITER 50
#endif
constexpr float kMprTol = MPCR_MPR_TOL;  // gap tolerance (oracle MPR_TOL); MuJoCo ccd_iterations cap below
constexpr int kMprIter = MPCR_MPR_ITER;
constexpr float kMprEps = 1.1920929e-07f;
__device__ __forceinline__ bool mpr_zero(float x) { return fabsf(x) < kMprEps; }

// Ties in the support mapping resolve as in the oracle's support(): a box /
// capsule / cylinder axis with |l_k| < kSupTie |l| contributes 0 (its face or
// segment centre: MuJoCo's mju_sign(0) = 0, widened to the fp32 rounding of a
// component that is exactly zero in fp64), and the hull climb moves to the
// neighbour that beats the current vertex the most (strictly; kSupBand > 0
// would make it the first within that many metres).
#ifndef MPCR_SUP_BAND
#define MPCR_SUP_BAND 0.f  // MuJoCo's strict climb (round 3; 1e-5 before)
#endif
#ifndef MPCR_SUP_TIE
#define MPCR_SUP_TIE 1e-6f  // < 0: MuJoCo's mju_sign (only an exact zero is a tie)
#endif
constexpr float kSupTie = MPCR_SUP_TIE;
// hull support ties (round 6, oracle HULL_TIE): vertices within this many
// metres of the climb's end are tied with it (hull_tie); 0 = the plain climb
#ifndef MPCR_HULL_TIE
#define MPCR_HULL_TIE 1e-7f
#endif
constexpr float kHullTie = MPCR_HULL_TIE;
constexpr float kSupBand = MPCR_SUP_BAND;
__device__ __forceinline__ float tie_sign(float lk, float ln) {
  if (kSupTie < 0.f) return lk > 0.f ? 1.f : (lk < 0.f ? -1.f : 0.f);
  return fabsf(lk) < kSupTie * ln ? 0.f : (lk >= 0.f ? 1.f : -1.f);
}

// examine the neighbours of vertex v along l (unit): one must beat bn (the
// current vertex + band, then the chosen neighbour + band); -1 if none.
// Neighbour records carry (index | degree << 16), so the next round's loads
// need no lookup: the first 8 neighbours (90 % of hull vertices have <= 8)
// sit in v's NaN-padded head block (addressed by v alone, 8 independent
// loads), the rest of a longer list in hull_adjv after one hull_info load.
// Hull support ties (round 6, the oracle's hull_tie): a round also keeps
// the lowest-index neighbour within kHullTie of the current vertex (tkey:
// index << 16 | degree, the record's w bits rotated; ~0u: none).  The round
// that ends the climb thus names the climb end's lowest tied neighbour, and
// sup_finish walks on to it while one is lower (tie_round).
__device__ __forceinline__ void climb_scan(const float4 (&w)[8], const float l[3], float& bn, float4& hv, int& nb,
                                           float lo, uint32_t& tkey) {
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const float du = w[j].x * l[0] + w[j].y * l[1] + w[j].z * l[2];  // NaN pads never win
    const uint32_t wb = __float_as_uint(w[j].w);
    if (du >= lo) tkey = min(tkey, __builtin_amdgcn_alignbit(wb, wb, 16));
    if (du > bn) { bn = du + kSupBand; nb = __float_as_int(w[j].w); hv = w[j]; }
  }
}
__device__ __forceinline__ int climb_round(const DevModel* __restrict__ m, int v, int deg, const float l[3],
                                           float& best, float4& hv, uint32_t& tkey) {
  int nb = -1;
  float bn = best + kSupBand;
  const float lo = best - kHullTie;
  tkey = ~0u;
  float4 w[8];
#pragma unroll
  for (int j = 0; j < 8; j++) w[j] = m->hull_head[(size_t)v * 8 + j];
  climb_scan(w, l, bn, hv, nb, lo, tkey);
  if (deg > 8) {
    const int a = m->hull_info[v].x, last = a + deg - 1;
    for (int k0 = a + 8; k0 <= last; k0 += 8) {
#pragma unroll
      for (int j = 0; j < 8; j++) w[j] = m->hull_adjv[min(k0 + j, last)];  // repeats of the last never win twice
      climb_scan(w, l, bn, hv, nb, lo, tkey);
    }
  }
  if (nb >= 0) best = bn - kSupBand;
  return nb;
}

// The support of a hull on a tie.  When the direction is normal (to
// ~kHullTie) to an edge or a face of the hull, every vertex of it is a
// maximum, and which one the climb reaches depends on where it started (the
// start table's cell, the pair's hint) and on the last bits of the dot
// products (fp32 and fp64 pick differently).  From the climb's end v the
// support walks to the lowest-index neighbour within kHullTie of v's value
// while that neighbour's index is lower: the tie's lowest index from
// whichever of its vertices the climb reached (the oracle's hull_tie), so a
// start table's resolution stays a performance choice, not a parity change
// (tests/test_hull_ties.py).  One walk round, out of line with scalar
// arguments (its call's spills stay on this path; inlined, or folded into
// the climb loop, the walk cost the hot climb registers or time): v's
// coordinates and the key of its lowest tied neighbour.
struct TieStep { float x, y, z; uint32_t tkey; };  // v's coordinates, its lowest tied neighbour's key
__device__ __noinline__ TieStep tie_round(const DevModel* __restrict__ m, int v, int deg, float lo, float l0,
                                          float l1, float l2) {
  uint32_t tkey = ~0u;
  const float l[3] = {l0, l1, l2};
  float4 w[8];
  const float4 x = m->hull_vert[v];
#pragma unroll
  for (int j = 0; j < 8; j++) w[j] = m->hull_head[(size_t)v * 8 + j];  // the head block's loads in flight together
  float bn = 3e38f;  // (no neighbour is climbed to)
  float4 hv;
  int nb;
  climb_scan(w, l, bn, hv, nb, lo, tkey);
  if (deg > 8) {
    const int a = m->hull_info[v].x, last = a + deg - 1;
    for (int k0 = a + 8; k0 <= last; k0 += 8) {
#pragma unroll
      for (int j = 0; j < 8; j++) w[j] = m->hull_adjv[min(k0 + j, last)];
      climb_scan(w, l, bn, hv, nb, lo, tkey);
    }
  }
  return TieStep{x.x, x.y, x.z, tkey};
}

// cube-map cell of a local direction (the engine's start table order,
// engine.hip hull_start_table; oracle lut_cell): major axis (lowest on ties), its sign, the other two components
// (cyclic order) over |l_axis| in MPCR_LUT_R bins
template <int R = MPCR_LUT_R>
__device__ __forceinline__ int lut_cell(const float l[3]) {
  const float a0 = fabsf(l[0]), a1 = fabsf(l[1]), a2 = fabsf(l[2]);
  const int ax = (a0 >= a1 && a0 >= a2) ? 0 : (a1 >= a2 ? 1 : 2);
  const float lax = ax == 0 ? l[0] : (ax == 1 ? l[1] : l[2]);
  const float lu = ax == 0 ? l[1] : (ax == 1 ? l[2] : l[0]);
  const float lv = ax == 0 ? l[2] : (ax == 1 ? l[0] : l[1]);
  const float la = fabsf(lax);
  if (!(la > 0.f)) return 0;
  const int iu = min(max((int)floorf((lu / la + 1.f) * 0.5f * R), 0), R - 1);
  const int iv = min(max((int)floorf((lv / la + 1.f) * 0.5f * R), 0), R - 1);
  return (2 * ax + (lax < 0.f ? 1 : 0)) * R * R + iu * R + iv;
}

// hint: hull vertex the previous query on this geom ended at (-1: none); the
// climb starts there (successive MPR directions are close)
// org (nullable): the result relative to org, with (geom centre - org)
// formed first -- MPR works relative to the second geom's centre, so the
// Minkowski points carry cm-scale rounding instead of world-scale (1 m) rounding
//
// A query runs in two parts so a caller can put two of them in flight
// together (MPR's support pair: round 5): sup_start issues the first loads
// of a mesh query -- the start table cell of the direction and the hint
// vertex, independent of each other (the hint's index is clamped to the
// hull: a query without one loads the hull's first vertex and ignores it) --
// and sup_finish consumes them: the hint if it beats the table vertex, then
// the climb (none from an exact cell, engine.hip).  Same values and
// comparisons as one call, so bitwise the same support point.
struct SupQ {
  float l[3], lu[3], ln;
  float4 hv, hh;
  int type, la;
};
// a geom's per-query constants (type, table, first hull vertex), loaded once
// per MPR run instead of in front of every support query (MPCR_SUP_GEOMQ)
#ifndef MPCR_SUP_GEOMQ
#define MPCR_SUP_GEOMQ 1
#endif
struct GeomQ { int type, la, h0; };
__device__ __forceinline__ GeomQ geom_q(const DevModel* __restrict__ m, int g) {
  GeomQ q{m->geom_type[g], m->geom_lutadr[g], m->geom_hulladr[g]};
  asm volatile("" : "+v"(q.type), "+v"(q.la), "+v"(q.h0));  // kept in registers, not re-loaded per query
  return q;
}
template <class S>
__device__ __forceinline__ void sup_start(const DevModel* __restrict__ m, const S& s, int g, const float dir[3],
                                          int hint, SupQ& q, const GeomQ* gq = nullptr) {
  const float* R = s.gxmat[g];
  mtv(q.l, R, dir);
  q.ln = sqrtf(dot3(q.l, q.l));
  q.type = gq ? gq->type : m->geom_type[g];
  if (q.type == 7) {
    const float il = q.ln > 0.f ? 1.f / q.ln : 0.f;
    q.lu[0] = q.l[0] * il; q.lu[1] = q.l[1] * il; q.lu[2] = q.l[2] * il;
    q.la = gq ? gq->la : m->geom_lutadr[g];
    const int h0 = gq ? gq->h0 : m->geom_hulladr[g];
    q.hv = q.la >= 0 ? m->hull_lut[q.la + lut_cell(q.l)] : m->hull_vert[h0];
    q.hh = m->hull_vert[hint >= 0 ? hint : h0];
  }
}
// MPCR_SAT_TIES 1: the SAT's value-only queries walk the ties too (A/B of
// the start independence, tools/scramble_check.py)
#ifndef MPCR_SAT_TIES
#define MPCR_SAT_TIES 0
#endif
template <class S>
// ties = false: the caller uses the support value only (the SAT's
// separations), which any tied vertex gives to within kHullTie
__device__ __forceinline__ void sup_finish(const DevModel* __restrict__ m, const S& s, int g, SupQ& q, float out[3],
                                           int& hint, const float* org, bool ties = true) {
  const float* R = s.gxmat[g];
  const float* sz = m->geom_size[g];
  const float* l = q.l;
  const float ln = q.ln;
  const int type = q.type;
  float p[3] = {0.f, 0.f, 0.f};
  if (type == 2 || type == 3) {  // sphere, capsule
    if (ln > 0.f) { p[0] = sz[0] * l[0] / ln; p[1] = sz[0] * l[1] / ln; p[2] = sz[0] * l[2] / ln; }
    if (type == 3) p[2] += tie_sign(l[2], ln) * sz[1];
  } else if (type == 5) {  // cylinder
    const float r = sqrtf(l[0] * l[0] + l[1] * l[1]);
    if (r > fmaxf(kSupTie, 0.f) * ln) { p[0] = sz[0] * l[0] / r; p[1] = sz[0] * l[1] / r; }
    p[2] = tie_sign(l[2], ln) * sz[1];
  } else if (type == 6) {  // box
    p[0] = tie_sign(l[0], ln) * sz[0];
    p[1] = tie_sign(l[1], ln) * sz[1];
    p[2] = tie_sign(l[2], ln) * sz[2];
  } else if (type == 7) {  // mesh hull: steepest ascent on the vertex graph
    // start: the table vertex of l's cube-map cell, or the hint (where the
    // previous query on this pair ended) when it beats that by the band
    const float* lu = q.lu;
    float4 hv = q.hv;
    const int hw = __float_as_int(hv.w);
    int v = q.la >= 0 ? (hw & 0x7fff) : m->geom_hulladr[g];
    if (!(q.la >= 0 && (hw & 0x8000))) {  // not an exact cell (engine.hip): the hint, then the climb
      int deg = q.la >= 0 ? (hw >> 16) : hw;
      float best = hv.x * lu[0] + hv.y * lu[1] + hv.z * lu[2];
      if (hint >= 0) {
        const float4 hh = q.hh;
        const float bh = hh.x * lu[0] + hh.y * lu[1] + hh.z * lu[2];
        // (on equal values the hint: after a tie walk it is the tie's lowest
        // index, so the climb then ends where it starts, with no walk)
        if (bh >= best + kSupBand) { v = hint; hv = hh; deg = __float_as_int(hh.w); best = bh; }
      }
      uint32_t tkey = ~0u;
      for (int guard = 0; guard < 4096; guard++) {
        PROF_COUNT(m, 19);
        const int nb = climb_round(m, v, deg, lu, best, hv, tkey);
        if (nb < 0) break;
        v = nb & 0xffff;
        deg = nb >> 16;
      }
      if (kHullTie > 0.f && ties && (int)(tkey >> 16) < v) {  // a lower-index tied neighbour: walk (hull_tie)
        const float lo = best - kHullTie;
        for (int guard = 0; guard < 64 && (int)(tkey >> 16) < v; guard++) {
          v = tkey >> 16;
          const TieStep ts = tie_round(m, v, tkey & 0xffff, lo, lu[0], lu[1], lu[2]);
          hv.x = ts.x; hv.y = ts.y; hv.z = ts.z;
          tkey = ts.tkey;
        }
      }
    }
    p[0] = hv.x; p[1] = hv.y; p[2] = hv.z;
    hint = v;
  }
  mv(out, R, p);
  if (org) {
    out[0] += s.gxpos[g][0] - org[0]; out[1] += s.gxpos[g][1] - org[1]; out[2] += s.gxpos[g][2] - org[2];
  } else {
    out[0] += s.gxpos[g][0]; out[1] += s.gxpos[g][1]; out[2] += s.gxpos[g][2];
  }
}
template <class S>
__device__ __forceinline__ void support_geom(const DevModel* __restrict__ m, const S& s, int g, const float dir[3],
                                             float out[3], int& hint, const float* org = nullptr, bool ties = true) {
  SupQ q;
  sup_start(m, s, g, dir, hint, q);
  sup_finish(m, s, g, q, out, hint, org, ties);
}

struct MprPt { float v[3], a[3], b[3]; };

template <class S>
__device__ __forceinline__ void mpr_support(const DevModel* __restrict__ m, const S& s, int g1, int g2,
                                            const float dir[3], MprPt& o, int (&hint)[2], float* trace = nullptr,
                                            const GeomQ* gq = nullptr) {
  const float nd[3] = {-dir[0], -dir[1], -dir[2]};
  SupQ q1, q2;  // both queries' first loads in flight together
  PROF_COUNT(m, 20);
  sup_start(m, s, g1, dir, hint[0], q1, gq);
  sup_start(m, s, g2, nd, hint[1], q2, gq ? gq + 1 : nullptr);
  sup_finish(m, s, g1, q1, o.a, hint[0], s.gxpos[g2]);  // relative to g2's centre
  sup_finish(m, s, g2, q2, o.b, hint[1], s.gxpos[g2]);
  o.v[0] = o.a[0] - o.b[0]; o.v[1] = o.a[1] - o.b[1]; o.v[2] = o.a[2] - o.b[2];
  if (trace) {
    const int q = (int)trace[47];
    if (q < 32) { trace[48 + 2 * q] = (float)hint[0]; trace[49 + 2 * q] = (float)hint[1]; trace[47] = (float)(q + 1); }
  }
}
__device__ __forceinline__ void nrm3(float v[3]) {
  const float n = sqrtf(dot3(v, v));
  if (n > 0.f) { v[0] /= n; v[1] /= n; v[2] /= n; }
}
__device__ __forceinline__ void mpr_dir(const MprPt p[4], float dir[3]) {
  float a[3] = {p[2].v[0] - p[1].v[0], p[2].v[1] - p[1].v[1], p[2].v[2] - p[1].v[2]};
  float b[3] = {p[3].v[0] - p[1].v[0], p[3].v[1] - p[1].v[1], p[3].v[2] - p[1].v[2]};
  cross(dir, a, b);
  nrm3(dir);
}
__device__ __forceinline__ bool mpr_reach(const MprPt p[4], const MprPt& v4, const float dir[3], float tol) {
  const float d4 = dot3(v4.v, dir);
  const float t = fminf(d4 - dot3(p[1].v, dir), fminf(d4 - dot3(p[2].v, dir), d4 - dot3(p[3].v, dir)));
  return t < tol;
}
__device__ __forceinline__ void mpr_expand(MprPt p[4], const MprPt& v4) {
  float x[3];
  cross(x, v4.v, p[0].v);
  if (dot3(p[1].v, x) > 0.f) {
    if (dot3(p[2].v, x) > 0.f) p[1] = v4; else p[3] = v4;
  } else {
    if (dot3(p[3].v, x) > 0.f) p[2] = v4; else p[1] = v4;
  }
}
__device__ __forceinline__ void tri_closest(const float a[3], const float b[3], const float c[3], float out[3]) {
  float ab[3], ac[3], ap[3], bp[3], cp[3];
#pragma unroll
  for (int k = 0; k < 3; k++) { ab[k] = b[k] - a[k]; ac[k] = c[k] - a[k]; ap[k] = -a[k]; bp[k] = -b[k]; cp[k] = -c[k]; }
  const float d1 = dot3(ab, ap), d2 = dot3(ac, ap);
  if (d1 <= 0.f && d2 <= 0.f) { out[0] = a[0]; out[1] = a[1]; out[2] = a[2]; return; }
  const float d3 = dot3(ab, bp), d4 = dot3(ac, bp);
  if (d3 >= 0.f && d4 <= d3) { out[0] = b[0]; out[1] = b[1]; out[2] = b[2]; return; }
  const float vc = d1 * d4 - d3 * d2;
  if (vc <= 0.f && d1 >= 0.f && d3 <= 0.f) {
    const float t = d1 / (d1 - d3);
    out[0] = a[0] + t * ab[0]; out[1] = a[1] + t * ab[1]; out[2] = a[2] + t * ab[2];
    return;
  }
  const float d5 = dot3(ab, cp), d6 = dot3(ac, cp);
  if (d6 >= 0.f && d5 <= d6) { out[0] = c[0]; out[1] = c[1]; out[2] = c[2]; return; }
  const float vb = d5 * d2 - d1 * d6;
  if (vb <= 0.f && d2 >= 0.f && d6 <= 0.f) {
    const float t = d2 / (d2 - d6);
    out[0] = a[0] + t * ac[0]; out[1] = a[1] + t * ac[1]; out[2] = a[2] + t * ac[2];
    return;
  }
  const float va = d3 * d6 - d5 * d4;
  if (va <= 0.f && (d4 - d3) >= 0.f && (d5 - d6) >= 0.f) {
    const float t = (d4 - d3) / ((d4 - d3) + (d5 - d6));
#pragma unroll
    for (int k = 0; k < 3; k++) out[k] = b[k] + t * (c[k] - b[k]);
    return;
  }
  // face region: the plane projection n (n.a) / |n|^2 (the oracle's
  // tri_closest): the barycentric a + v ab + w ac cancels catastrophically in
  // fp32 for MPR's cm-sized final portal around a sub-mm penetration
  float n[3];
  cross(n, ab, ac);
  const float sc = dot3(n, a) / dot3(n, n);
#pragma unroll
  for (int k = 0; k < 3; k++) out[k] = n[k] * sc;
  (void)va; (void)vb; (void)vc;
}

// returns true and (depth, dir g1 -> g2, pos) when the geoms overlap.
// Zero tests are geometric and in metres, identical in the oracle: libccd's
// are absolute DBL_EPSILON tests on lengths, areas and volumes alike, which
// in fp32 call two cm-scale vectors parallel (|v0 x v1|^2 ~ 1e-8 < eps);
// here a length is zero below kMprEps (1.2e-7 m, fp32 resolution of world
// coordinates), two vectors are parallel when one passes within kMprEps of
// the other's line, and a point lies on a plane within kMprEps of it.
template <class S>
__device__ bool mpr_lane(const DevModel* __restrict__ m, const S& s, int g1, int g2, float& depth, float dir[3],
                         float pos[3], int (&hint)[2], float* trace = nullptr) {
  MprPt p[4], v4;
  float va[3], vb[3], dd;
  const float tol = kMprTol;
#if MPCR_SUP_GEOMQ
  const GeomQ gqa[2] = {geom_q(m, g1), geom_q(m, g2)};
  const GeomQ* const gq = gqa;
#else
  const GeomQ* const gq = nullptr;
#endif
  // point x off the plane through the origin with (unnormalised) normal c by more than kMprEps
  auto off_plane = [](float x, const float c[3]) { return fabsf(x) >= kMprEps * sqrtf(dot3(c, c)); };
#pragma unroll
  for (int k = 0; k < 3; k++) {  // the frame of the Minkowski points: origin at g2's centre
    p[0].a[k] = s.gxpos[g1][k] - s.gxpos[g2][k];
    p[0].b[k] = 0.f;
    p[0].v[k] = p[0].a[k];
  }
  if (mpr_zero(p[0].v[0]) && mpr_zero(p[0].v[1]) && mpr_zero(p[0].v[2])) p[0].v[0] += 10.f * kMprEps;
  dir[0] = -p[0].v[0]; dir[1] = -p[0].v[1]; dir[2] = -p[0].v[2];
  nrm3(dir);
  mpr_support(m, s, g1, g2, dir, p[1], hint, trace, gq);
  dd = dot3(p[1].v, dir);
  if (mpr_zero(dd) || dd < 0.f) return false;
  cross(dir, p[0].v, p[1].v);
  {
    const float thr = kMprEps * (sqrtf(dot3(p[0].v, p[0].v)) + sqrtf(dot3(p[1].v, p[1].v)));
    if (dot3(dir, dir) < thr * thr) {  // v1 on the ray from v0 through the origin
#pragma unroll
      for (int k = 0; k < 3; k++) pos[k] = 0.5f * (p[1].a[k] + p[1].b[k]) + s.gxpos[g2][k];
      if (mpr_zero(p[1].v[0]) && mpr_zero(p[1].v[1]) && mpr_zero(p[1].v[2])) {
        depth = 0.f;
        dir[0] = dir[1] = dir[2] = 0.f;
      } else {
        dir[0] = p[1].v[0]; dir[1] = p[1].v[1]; dir[2] = p[1].v[2];
        depth = sqrtf(dot3(dir, dir));
        nrm3(dir);
      }
      return true;
    }
  }
  nrm3(dir);
  mpr_support(m, s, g1, g2, dir, p[2], hint, trace, gq);
  dd = dot3(p[2].v, dir);
  if (mpr_zero(dd) || dd < 0.f) return false;
#pragma unroll
  for (int k = 0; k < 3; k++) { va[k] = p[1].v[k] - p[0].v[k]; vb[k] = p[2].v[k] - p[0].v[k]; }
  cross(dir, va, vb);
  nrm3(dir);
  if (dot3(dir, p[0].v) > 0.f) {
    const MprPt t = p[1]; p[1] = p[2]; p[2] = t;
    dir[0] = -dir[0]; dir[1] = -dir[1]; dir[2] = -dir[2];
  }
  for (int guard = 0;; guard++) {
    if (guard > kMprIter) return false;
    mpr_support(m, s, g1, g2, dir, p[3], hint, trace, gq);
    dd = dot3(p[3].v, dir);
    if (mpr_zero(dd) || dd < 0.f) return false;
    bool cont = false;
    cross(va, p[1].v, p[3].v);
    dd = dot3(va, p[0].v);
    if (dd < 0.f && off_plane(dd, va)) { p[2] = p[3]; cont = true; }
    if (!cont) {
      cross(va, p[3].v, p[2].v);
      dd = dot3(va, p[0].v);
      if (dd < 0.f && off_plane(dd, va)) { p[1] = p[3]; cont = true; }
    }
    if (trace) trace[9] = (float)guard;
    if (!cont) break;
#pragma unroll
    for (int k = 0; k < 3; k++) { va[k] = p[1].v[k] - p[0].v[k]; vb[k] = p[2].v[k] - p[0].v[k]; }
    cross(dir, va, vb);
    nrm3(dir);
  }
  for (int it = 0;; it++) {
    if (trace) trace[10] = (float)it;
    mpr_dir(p, dir);
    dd = dot3(dir, p[1].v);
    if (mpr_zero(dd) || dd > 0.f) break;
    mpr_support(m, s, g1, g2, dir, v4, hint, trace, gq);
    dd = dot3(v4.v, dir);
    if (!(mpr_zero(dd) || dd > 0.f) || mpr_reach(p, v4, dir, tol) || it > kMprIter) return false;
    mpr_expand(p, v4);
  }
  for (int it = 0;; it++) {
    if (trace) trace[11] = (float)it;
    mpr_dir(p, dir);
    mpr_support(m, s, g1, g2, dir, v4, hint, trace, gq);
    if (mpr_reach(p, v4, dir, tol) || it > kMprIter) break;
    mpr_expand(p, v4);
  }
  if (trace)
    for (int i = 0; i < 4; i++)
      for (int k = 0; k < 3; k++) {
        trace[12 + 9 * i + k] = p[i].v[k];
        trace[12 + 9 * i + 3 + k] = p[i].a[k];
        trace[12 + 9 * i + 6 + k] = p[i].b[k];
      }
  float w[3];
  tri_closest(p[1].v, p[2].v, p[3].v, w);
  depth = sqrtf(dot3(w, w));
  if (mpr_zero(depth)) { dir[0] = dir[1] = dir[2] = 0.f; }
  else { dir[0] = w[0] / depth; dir[1] = w[1] / depth; dir[2] = w[2] / depth; }
  float pd[3], b[4], x[3];
  {
    float e1[3] = {p[2].v[0] - p[1].v[0], p[2].v[1] - p[1].v[1], p[2].v[2] - p[1].v[2]};
    float e2[3] = {p[3].v[0] - p[1].v[0], p[3].v[1] - p[1].v[1], p[3].v[2] - p[1].v[2]};
    cross(pd, e1, e2);  // portal normal, |pd| = twice the portal's area
  }
  cross(x, p[2].v, p[3].v); b[0] = dot3(x, p[1].v);
  cross(x, p[3].v, p[2].v); b[1] = dot3(x, p[0].v);
  cross(x, p[0].v, p[1].v); b[2] = dot3(x, p[3].v);
  cross(x, p[2].v, p[1].v); b[3] = dot3(x, p[0].v);
  float sum = b[0] + b[1] + b[2] + b[3];
  // sum = 6 x the tetrahedron's volume: degenerate when v0 lies within kMprEps of the portal's plane
  if (!off_plane(sum, pd) || sum < 0.f) {
    nrm3(pd);
    b[0] = 0.f;
    cross(x, p[2].v, p[3].v); b[1] = dot3(x, pd);
    cross(x, p[3].v, p[1].v); b[2] = dot3(x, pd);
    cross(x, p[1].v, p[2].v); b[3] = dot3(x, pd);
    sum = b[1] + b[2] + b[3];
  }
#pragma unroll
  for (int k = 0; k < 3; k++) {
    float pa = 0.f, pb = 0.f;
#pragma unroll
    for (int i = 0; i < 4; i++) { pa += b[i] * p[i].a[k]; pb += b[i] * p[i].b[k]; }
    pos[k] = 0.5f * (pa + pb) / sum + s.gxpos[g2][k];
  }
  return true;
}

__device__ __forceinline__ bool beats(float v, float best) { return v > best + 1e-4f * fabsf(best) + 1e-12f; }
__device__ __forceinline__ bool near_max(float v, float mx) { return v >= mx - (1e-4f * fabsf(mx) + 1e-12f); }
__device__ __forceinline__ float wmax(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// inline the manifold callees (experiment): 1 polyhedron, 2 both
#ifndef MPCR_POLY_INLINE
#define MPCR_POLY_INLINE 2  // both inlined: 241 -> 235 VGPRs, no scratch (the contact arrays stay in registers), C4 48.6 -> 46.7 ms
#endif
// Plane-mesh manifold (MJX plane_convex / _manifold_points, the oracle's
// col_plane_mesh), wave-cooperative: every lane calls it with the same pair
// (mesh g, plane normal n through xp, penetration depth) and lane q receives
// the contacts.  The hull's vertices are scanned 64 at a time -- a first /
// last ballot for the penetrating set, then per pick a wave max and a ballot
// for its first index within the tie band (near_max, as the oracle) -- instead
// of four serial per-lane scans (a 2691-vertex hull touching the table made a
// handful of dual-arm candidates 3x slower than the rest).
template <class S>
#if MPCR_POLY_INLINE >= 2
__device__ __forceinline__
#else
__device__ __noinline__
#endif
void plane_mesh_manifold_wave(const DevModel* __restrict__ m_, const S& s, int g,
                                                      const float n_[3], const float* xp_, float depth, int q, int lane,
                                                      float dist[4], float pos[4][3], float nrm[4][3], int& nsl) {
  const MPCR_GMEM DevModel* __restrict__ m = uniform_model(m_);
  ASSUME_LDS(&s); ASSUME_PRIVATE(dist); ASSUME_PRIVATE(pos); ASSUME_PRIVATE(nrm); ASSUME_PRIVATE(&nsl);
  const float n[3] = {n_[0], n_[1], n_[2]}, xp[3] = {xp_[0], xp_[1], xp_[2]};  // in registers (no alias reloads)
  const float* R = s.gxmat[g];
  const float* xg = s.gxpos[g];
  float nl[3], pl[3];
  mtv(nl, R, n);
  const float dx[3] = {xp[0] - xg[0], xp[1] - xg[1], xp[2] - xg[2]};
  mtv(pl, R, dx);
  const float thr = fmaxf(0.f, depth - 1e-3f);
  const int v0 = m->geom_hulladr[g], v1 = v0 + m->geom_hullnum[g];
  const MPCR_GMEM float4* __restrict__ hv = m->hull_vert;
  auto sup = [&](const float4& v) { return (pl[0] - v.x) * nl[0] + (pl[1] - v.y) * nl[1] + (pl[2] - v.z) * nl[2]; };
  int ia = -1, il = -1;
  for (int base = v0; base < v1; base += WAVE) {
    const int i = base + lane;
    const unsigned long long bm = __ballot(i < v1 && sup(hv[i < v1 ? i : v0]) > thr);
    if (bm) {
      if (ia < 0) ia = base + __builtin_ctzll(bm);
      il = base + 63 - __builtin_clzll(bm);
    }
  }
  if (ia < 0) {  // the climb's vertex alone (threshold rounding): lane q keeps it
    if (lane == q) nsl = 1;
    return;
  }
  // max of e over the penetrating set, then its first index within the band
  auto pick = [&](auto&& ef, float& mx) {
    float lm = -1.f;
    for (int base = ia; base <= il; base += WAVE) {
      const int i = base + lane;
      if (i <= il) {
        const float4 v = hv[i];
        if (sup(v) > thr) lm = fmaxf(lm, ef(v));
      }
    }
    mx = wmax(lm);
    for (int base = ia; base <= il; base += WAVE) {
      const int i = base + lane;
      bool hit = false;
      if (i <= il) {
        const float4 v = hv[i];
        hit = sup(v) > thr && near_max(ef(v), mx);
      }
      const unsigned long long bm = __ballot(hit);
      if (bm) return base + __builtin_ctzll(bm);
    }
    return ia;  // unreachable: the maximum itself is within the band
  };
  const float4 a = hv[ia];
  float mx;
  const int ib = pick([&](const float4& v) {
    return (a.x - v.x) * (a.x - v.x) + (a.y - v.y) * (a.y - v.y) + (a.z - v.z) * (a.z - v.z);
  }, mx);
  const float4 b = hv[ib];
  float ab[3];
  {
    const float amb[3] = {a.x - b.x, a.y - b.y, a.z - b.z};
    cross(ab, nl, amb);
  }
  const int ic = pick([&](const float4& v) {
    return fabsf((a.x - v.x) * ab[0] + (a.y - v.y) * ab[1] + (a.z - v.z) * ab[2]);
  }, mx);
  const float4 c = hv[ic];
  float ac[3], bc[3];
  {
    const float amc[3] = {a.x - c.x, a.y - c.y, a.z - c.z}, bmc[3] = {b.x - c.x, b.y - c.y, b.z - c.z};
    cross(ac, nl, amc);
    cross(bc, nl, bmc);
  }
  float bbp, bap;
  const int ibp = pick([&](const float4& v) {
    return fabsf((b.x - v.x) * bc[0] + (b.y - v.y) * bc[1] + (b.z - v.z) * bc[2]);
  }, bbp);
  const int iap = pick([&](const float4& v) {
    return fabsf((a.x - v.x) * ac[0] + (a.y - v.y) * ac[1] + (a.z - v.z) * ac[2]);
  }, bap);
  const int idx[4] = {ia, ib, ic, beats(bap, bbp) ? iap : ibp};
#pragma unroll
  for (int k = 0; k < 4; k++) {
    bool dup = false;
#pragma unroll
    for (int t = 0; t < k; t++) dup |= idx[t] == idx[k];
    const float4 v = hv[idx[k]];
    const float l[3] = {v.x, v.y, v.z};
    float w[3];
    mv(w, R, l);
    const float d = -sup(v);
    if (lane == q) {
      dist[k] = dup ? 1e30f : d;
#pragma unroll
      for (int e = 0; e < 3; e++) { pos[k][e] = w[e] + xg[e] - 0.5f * d * n[e]; nrm[k][e] = n[e]; }
    }
  }
  if (lane == q) nsl = 4;
}

constexpr int kPendingManifold = -4;  // narrow_lane: plane-mesh pair awaiting plane_mesh_manifold_wave
constexpr float kPolyConeCos = 0.94f;  // ~20 degrees: candidate faces' Gauss-map cone about MPR's normal
static_assert(kPolyConeCos == (float)CONE_COS, "the host's cone table is built for this cone");
constexpr int kPendingPoly = -5;      // narrow_lane: polyhedron pair hit by MPR, awaiting poly_manifold_wave

// hull vertex index of geom g's support point along dir (world): the mesh
// climb from hint (the pair's, read only), or the box corner (+ side on an
// exactly zero component) -- the oracle's support_vertex
template <class S>
__device__ __forceinline__ int support_vertex(const DevModel* __restrict__ m, const S& s, int g, const float dir[3],
                                              int hint) {
  if (m->geom_type[g] == 6) {
    // the corner on the side of each axis; an axis within the tie band of
    // zero (a face normal from fp32 rounding) takes the + side, as MPR's box
    // support does (tie_sign)
    float l[3];
    mtv(l, s.gxmat[g], dir);
    const float ln = sqrtf(l[0] * l[0] + l[1] * l[1] + l[2] * l[2]);
    return m->geom_cornadr[g] + (tie_sign(l[0], ln) >= 0.f ? 1 : 0) + (tie_sign(l[1], ln) >= 0.f ? 2 : 0) +
           (tie_sign(l[2], ln) >= 0.f ? 4 : 0);
  }
  float p[3];
  support_geom(m, s, g, dir, p, hint);
  return hint;
}

// world outward normal of face f of geom g and its plane offset relative to
// c (nw . (x - c) = off on the face)
template <class S>
__device__ __forceinline__ void face_rel_fp(const S& s, int g, const float4 fp, const float* c, float nw[3],
                                            float& off) {
  const float nl[3] = {fp.x, fp.y, fp.z};
  mv(nw, s.gxmat[g], nl);
  off = fp.w + nw[0] * (s.gxpos[g][0] - c[0]) + nw[1] * (s.gxpos[g][1] - c[1]) + nw[2] * (s.gxpos[g][2] - c[2]);
}
template <class S>
__device__ __forceinline__ void face_rel(const DevModel* __restrict__ m, const S& s, int g, int f, const float* c,
                                         float nw[3], float& off) {
  const float4 fp = m->face_plane[f];
  const float nl[3] = {fp.x, fp.y, fp.z};
  mv(nw, s.gxmat[g], nl);
  off = fp.w + nw[0] * (s.gxpos[g][0] - c[0]) + nw[1] * (s.gxpos[g][1] - c[1]) + nw[2] * (s.gxpos[g][2] - c[2]);
}

// hull vertex v of geom g relative to c
template <class S>
__device__ __forceinline__ void vert_rel(const DevModel* __restrict__ m, const S& s, int g, int v, const float* c,
                                         float w[3]) {
  const float4 hv = m->hull_vert[v];
  const float l[3] = {hv.x, hv.y, hv.z};
  mv(w, s.gxmat[g], l);
  w[0] += s.gxpos[g][0] - c[0]; w[1] += s.gxpos[g][1] - c[1]; w[2] += s.gxpos[g][2] - c[2];
}

// Polyhedron pairs (mesh-mesh, box-mesh): the face-clipping manifold
// (mujoco-mjx 3.3.1 convex_convex; the oracle's poly_manifold, same rules and
// orders), wave-cooperative: every lane calls it with the same pair and MPR's
// normal n (g1 -> g2) / depth, lane q receives up to 4 contacts (nsl = 4) or
// keeps MPR's single one (nsl = 1: an edge axis carries the contact).  One
// lane per candidate reference face (the faces on both support vertices and
// those within the Gauss-map cone of MPR's normal) with its own support query
// for the SAT separation, one lane per candidate
// incident face, Sutherland-Hodgman against the reference face's side planes
// with one lane per polygon vertex and scan compaction (as box_box_wave), the
// _manifold_points picks as wave maxima.  Coordinates relative to g2's
// centre, as MPR's.
// PS: the clip polygon / SAT-separation scratch (polyw, satsep): the LDS
// image's own, or -- the second wave of a two-wave candidate in the joint
// convex flush -- a PolyScratchT in the dead dynamics region.
template <class S, class PS>
#if MPCR_POLY_INLINE
__device__ __forceinline__
#else
__device__ __noinline__
#endif
void poly_manifold_wave(const DevModel* __restrict__ m_, const S& s, PS& ps, const short* hints, int p,
                                                const float n_[3], float depth, int q, int lane, float dist[4],
                                                float pos[4][3], float nrm[4][3], int& nsl) {
  const MPCR_GMEM DevModel* __restrict__ m = uniform_model(m_);
  ASSUME_GLOBAL(hints); ASSUME_LDS(&s); ASSUME_LDS(&ps); ASSUME_PRIVATE(dist); ASSUME_PRIVATE(pos); ASSUME_PRIVATE(nrm);
  ASSUME_PRIVATE(&nsl);
  const float n[3] = {n_[0], n_[1], n_[2]};  // in registers (no alias reloads)
  PSTAMP_DECL
  const int g1 = m->pair_g1[p], g2 = m->pair_g2[p];
  const float c[3] = {s.gxpos[g2][0], s.gxpos[g2][1], s.gxpos[g2][2]};
  const int hw = reinterpret_cast<const int*>(hints)[p - m->cvx_base];
  const int h0 = (int)(short)(hw & 0xffff), h1 = hw >> 16;
  // support vertices: lane 0 of g1 along n, lane 1 of g2 along -n
  int sv = 0;
  if (lane < 2) {
    const float sg = lane ? -1.f : 1.f;
    const float d[3] = {sg * n[0], sg * n[1], sg * n[2]};
    sv = support_vertex(m, s, lane ? g2 : g1, d, lane ? h1 : h0);
  }
  const int s1 = __shfl(sv, 0), s2 = __shfl(sv, 1);
  PSTAMP(m, 23);
  const int2 i1 = m->vert_finfo[s1], i2 = m->vert_finfo[s2];
  // a deep penetration between small hulls: every face is a candidate (MPR's
  // normal, which seeds the cone below, is that deep the portal face MPR
  // ended on -- fp32 and fp64 ended 70 degrees apart on the Hand-E's
  // interpenetrating finger pads)
  const int nf1 = m->geom_facenum[g1], nf2 = m->geom_facenum[g2];
  const bool allf = POLY_ALLF_ON && depth > POLY_DEEP && nf1 + nf2 <= POLY_ALLF;
  float bsep = 0.f;
  int fr = -1;
  bool rtwo = false, found = false;
  if (allf) {
    // SAT separation of every face (lane = face, rounds of 64) into LDS,
    // the wave max, then the lowest face index within the max's tie band
    // (MPCR_ALLF_U faces per lane per pass: their face-plane loads, then
    // their support queries' first loads, in flight together -- a pass was
    // two dependent load latencies per 64 faces, up to 8 passes in turn)
    const int fa1 = m->geom_faceadr[g1], fa2 = m->geom_faceadr[g2], nf = nf1 + nf2;
    constexpr int U = MPCR_ALLF_U;
    float mxl = -3e38f;  // this lane's maximum (the wave max below: max is exact in any order)
#pragma unroll 1
    for (int b0 = 0; b0 < nf; b0 += U * WAVE) {
      float4 fp[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int k = b0 + u * WAVE + lane;
        fp[u] = make_float4(0.f, 0.f, 1.f, 0.f);
        if (k < nf) fp[u] = m->face_plane[k >= nf1 ? fa2 + k - nf1 : fa1 + k];
      }
      SupQ q[U];
      float nw[U][3], off[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int k = b0 + u * WAVE + lane;
        if (k < nf) {
          const bool two = k >= nf1;
          const int g = two ? g2 : g1, go = two ? g1 : g2;
          face_rel_fp(s, g, fp[u], c, nw[u], off[u]);
          const float mn[3] = {-nw[u][0], -nw[u][1], -nw[u][2]};
          sup_start(m, s, go, mn, two ? h0 : h1, q[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int k = b0 + u * WAVE + lane;
        if (k < nf) {
          const bool two = k >= nf1;
          float pt[3];
          int h = two ? h0 : h1;
          sup_finish(m, s, two ? g1 : g2, q[u], pt, h, c, MPCR_SAT_TIES != 0);
          const float sp = nw[u][0] * pt[0] + nw[u][1] * pt[1] + nw[u][2] * pt[2] - off[u];
          ps.satsep[k] = sp;
          mxl = fmaxf(mxl, sp);
        }
      }
    }
    const float mxa = wmax(mxl);
    sync();
    // the key 2 f + side keeps the side with the face: two geoms of one mesh
    // share their face range, and on equal faces g1's wins, the
    // oracle's first-listed candidate
    float fmin = 3e38f;
#pragma unroll 1
    for (int b0 = 0; b0 < nf; b0 += WAVE) {
      const int k = b0 + lane;
      const bool nb = k < nf && near_max(ps.satsep[k], mxa);
      const int key = k >= nf1 ? 2 * (fa2 + k - nf1) + 1 : 2 * (fa1 + k);
      fmin = fminf(fmin, -wmax(nb ? -(float)key : -3e38f));
    }
    found = fmin < 3e38f;
    if (found) {
      const int key = (int)fmin;
      fr = key >> 1;
      rtwo = (key & 1) != 0;
      bsep = ps.satsep[rtwo ? nf1 + fr - fa2 : fr - fa1];
    }
    sync();  // satsep shares bytes with the clip buffer below
  }
  const int c1 = allf ? 0 : min(i1.y, WAVE), c2 = allf ? 0 : min(i2.y, WAVE - c1), ns = c1 + c2;
  // candidate reference faces, at most 64 (one per lane), in the oracle's
  // order: g1's on s1, g2's on s2, then every face whose outward normal lies
  // within the Gauss-map cone of n (g1) / -n (g2), face index order, those
  // already listed skipped -- a ballot-compacted scan of both face tables into
  // an LDS list (the clip buffer's second half, free until the clip)
  // The faces scanned are the host's cone table entries for the cube-map cell
  // of the local direction (DevModel::cone_cell: a superset of the faces the
  // test below accepts, ascending), not all of the geom's faces (up to 5219
  // on the dual arm's hulls): the same candidates in the same order.  The
  // support-vertex faces of each side sit one per lane (lane k: entry k) and
  // the duplicate test reads them with readlane.
  int* const cl = reinterpret_cast<int*>(&ps.polyw[1][0][0]);
  int nc = ns;
  const int vf1 = lane < c1 ? m->vert_face[i1.x + lane] : -1, vf2 = lane < c2 ? m->vert_face[i2.x + lane] : -1;
#pragma unroll 1
  for (int sd = 0; sd < 2 && !allf; sd++) {
    const int g = sd ? g2 : g1;
    const int cs = sd ? c2 : c1, vfs = sd ? vf2 : vf1;
    const float sg = sd ? -1.f : 1.f;
    float l[3];
    {
      const float dn[3] = {sg * n[0], sg * n[1], sg * n[2]};
      mtv(l, s.gxmat[g], dn);
    }
    const int2 cc = m->cone_cell[m->geom_coneadr[g] + lut_cell<CONE_R>(l)];
#pragma unroll 1
    for (int b0 = 0; b0 < cc.y && nc < WAVE; b0 += WAVE) {
      bool sel = false;
      int f = -1;
      if (b0 + lane < cc.y) {
        f = m->cone_face[cc.x + b0 + lane];
        const float4 fp = m->face_plane[f];
        const float nl[3] = {fp.x, fp.y, fp.z};
        float nw[3];
        mv(nw, s.gxmat[g], nl);
        sel = sg * (nw[0] * n[0] + nw[1] * n[1] + nw[2] * n[2]) >= kPolyConeCos;
      }
#pragma unroll 1
      for (int k = 0; k < cs; k++) sel &= __builtin_amdgcn_readlane(vfs, k) != f;
      int tot;
      const int o = wscan_excl(sel ? 1 : 0, tot);
      if (sel && nc + o < WAVE) cl[nc - ns + o] = f | (sd << 24);
      nc = min(nc + tot, WAVE);
    }
  }
  sync();
  PSTAMP(m, 24);
  // SAT separation along each candidate's outward normal
  float sep = -3e38f;
  int fid = -1, two = 0;
  if (!allf && lane < nc) {
    if (lane < ns) {
      two = lane >= c1;
      fid = m->vert_face[two ? i2.x + lane - c1 : i1.x + lane];
    } else {
      const int e = cl[lane - ns];
      two = e >> 24;
      fid = e & 0xffffff;
    }
    const int g = two ? g2 : g1, go = two ? g1 : g2;
    float nw[3], off, pt[3];
    face_rel(m, s, g, fid, c, nw, off);
    const float mn[3] = {-nw[0], -nw[1], -nw[2]};
    int h = two ? h0 : h1;
    support_geom(m, s, go, mn, pt, h, c, MPCR_SAT_TIES != 0);
    sep = nw[0] * pt[0] + nw[1] * pt[1] + nw[2] * pt[2] - off;
  }
  // the maximum's tie band: the lowest face index (a flush face pair has the
  // same separation from either side)
  if (!allf) {
    const float mx = wmax(sep);
    const bool nb = lane < nc && near_max(sep, mx);
    const float fmn = -wmax(nb ? -(float)fid : -3e38f);
    const unsigned long long bm = __ballot(nb && (float)fid == fmn);
    const int kb = bm ? __builtin_ctzll(bm) : 0;
    found = bm != 0;
    bsep = __shfl(sep, kb);
    fr = __shfl(fid, kb);
    rtwo = __shfl(two, kb) != 0;
  }
  PSTAMP(m, 25);
  if (!found || -bsep > 1.05f * depth + 1e-5f) {  // an edge axis: MPR's single contact
    if (lane == q) nsl = 1;
    return;
  }
  const int gr = rtwo ? g2 : g1, gi = rtwo ? g1 : g2;
  float nr[3], offr;
  face_rel(m, s, gr, fr, c, nr, offr);
  // the reference polygon's vertices (lane k: vertex k), loaded here so their
  // latency hides behind the incident face's support climb
  const int2 fri = m->face_vinfo[fr];
  const int nrv = fri.y;
  float A[3] = {0.f, 0.f, 0.f}, sn[3];
  if (lane < nrv) vert_rel(m, s, gr, m->face_vert[fri.x + lane], c, A);
  // incident face: the most anti-parallel face on gi's support vertex along -nr
  int si = 0;
  if (lane == 0) {
    const float d[3] = {-nr[0], -nr[1], -nr[2]};
    si = support_vertex(m, s, gi, d, rtwo ? h0 : h1);
  }
  si = __shfl(si, 0);
  const int2 ii = m->vert_finfo[si];
  const int ci = min(ii.y, WAVE);
  float al = -3e38f;
  int finc = -1;
  if (lane < ci) {
    finc = m->vert_face[ii.x + lane];
    const float4 fp = m->face_plane[finc];
    const float nl[3] = {fp.x, fp.y, fp.z};
    float nw[3];
    mv(nw, s.gxmat[gi], nl);
    al = -(nw[0] * nr[0] + nw[1] * nr[1] + nw[2] * nr[2]);
  }
  const float mxa = wmax(al);
  const unsigned long long bma = __ballot(lane < ci && near_max(al, mxa));
  if (!bma) {
    if (lane == q) nsl = 1;
    return;
  }
  const int fi = __shfl(finc, __builtin_ctzll(bma));
  // reference polygon (lane k: vertex k and its edge's outward side-plane
  // normal), incident polygon into the clip buffer
  const int2 fii = m->face_vinfo[fi];
  const int ninc = fii.y;
  {
    const int ln = lane + 1 >= nrv ? 0 : lane + 1;
    const float ed[3] = {__shfl(A[0], ln) - A[0], __shfl(A[1], ln) - A[1], __shfl(A[2], ln) - A[2]};
    cross(sn, ed, nr);
  }
  if (lane < ninc) {
    float w[3];
    vert_rel(m, s, gi, m->face_vert[fii.x + lane], c, w);
    ps.polyw[0][lane][0] = w[0]; ps.polyw[0][lane][1] = w[1]; ps.polyw[0][lane][2] = w[2];
  }
  sync();
  PSTAMP(m, 26);
  int np = ninc, cur = 0;
  for (int e = 0; e < nrv && np > 0; e++) {
    const float Ae[3] = {__shfl(A[0], e), __shfl(A[1], e), __shfl(A[2], e)};
    const float se[3] = {__shfl(sn[0], e), __shfl(sn[1], e), __shfl(sn[2], e)};
    float P[3] = {0.f, 0.f, 0.f}, Q[3] = {0.f, 0.f, 0.f}, dp = 0.f, dq = 0.f;
    int e0 = 0, e1 = 0;
    if (lane < np) {
      const int k2 = lane + 1 == np ? 0 : lane + 1;
#pragma unroll
      for (int k = 0; k < 3; k++) { P[k] = ps.polyw[cur][lane][k]; Q[k] = ps.polyw[cur][k2][k]; }
      dp = se[0] * (P[0] - Ae[0]) + se[1] * (P[1] - Ae[1]) + se[2] * (P[2] - Ae[2]);
      dq = se[0] * (Q[0] - Ae[0]) + se[1] * (Q[1] - Ae[1]) + se[2] * (Q[2] - Ae[2]);
      e0 = dp <= 0.f;
      e1 = (dp < 0.f && dq > 0.f) || (dp > 0.f && dq < 0.f);
    }
    int tot;
    const int o = wscan_excl(e0 + e1, tot);
    if (e0 && o < S::PMAXW) {
#pragma unroll
      for (int k = 0; k < 3; k++) ps.polyw[cur ^ 1][o][k] = P[k];
    }
    if (e1 && o + e0 < S::PMAXW) {
      const float wgt = dp / (dp - dq);
#pragma unroll
      for (int k = 0; k < 3; k++) ps.polyw[cur ^ 1][o + e0][k] = P[k] + wgt * (Q[k] - P[k]);
    }
    np = min(tot, S::PMAXW);
    cur ^= 1;
    sync();
  }
  // the clipped points below the reference plane
  float P[3] = {0.f, 0.f, 0.f}, dk = 3e38f;
  bool keep = false;
  if (lane < np) {
#pragma unroll
    for (int k = 0; k < 3; k++) P[k] = ps.polyw[cur][lane][k];
    dk = nr[0] * P[0] + nr[1] * P[1] + nr[2] * P[2] - offr;
    keep = dk < m->pair_margin[p];
  }
  const unsigned long long km = __ballot(keep);
  const int nk = __popcll(km);
  sync();  // the clip buffer is free for the next pair
  PSTAMP(m, 27);
  const float sg = rtwo ? -1.f : 1.f;  // contact normal g1 -> g2
  if (nk == 0) {
    // no clipped point below the reference plane (a small reference face
    // over a deep penetration): the SAT axis still carries the contact, one
    // point at gi's support vertex along -nr (the oracle's rule; MPR's own
    // normal for a penetration this deep is path-dependent)
    float w[3];
    vert_rel(m, s, gi, si, c, w);
    const float dk = nr[0] * w[0] + nr[1] * w[1] + nr[2] * w[2] - offr;
    if (lane == q) {
      if (dk < m->pair_margin[p]) {
        dist[0] = dk;
        dist[1] = dist[2] = dist[3] = 1e30f;
#pragma unroll
        for (int e = 0; e < 3; e++) { pos[0][e] = w[e] - 0.5f * dk * nr[e] + c[e]; nrm[0][e] = sg * nr[e]; }
        nsl = 4;
      } else {
        nsl = 1;
      }
    }
    return;
  }
  int idx[4] = {-1, -1, -1, -1};
  if (nk <= 4) {
    unsigned long long r = km;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (r) { idx[j] = __builtin_ctzll(r); r &= r - 1; }
    }
  } else {
    // _manifold_points: a = the first, b = the farthest from a, c = the
    // farthest from line ab, d = the farthest from edge bc or ac
    auto pick = [&](float e, float& mxv) {
      mxv = wmax(keep ? e : -1.f);
      return __builtin_ctzll(__ballot(keep && near_max(e, mxv)));
    };
    const int ia = __builtin_ctzll(km);
    const float a[3] = {__shfl(P[0], ia), __shfl(P[1], ia), __shfl(P[2], ia)};
    float mxv;
    const int ib = pick((a[0] - P[0]) * (a[0] - P[0]) + (a[1] - P[1]) * (a[1] - P[1]) + (a[2] - P[2]) * (a[2] - P[2]),
                        mxv);
    const float b[3] = {__shfl(P[0], ib), __shfl(P[1], ib), __shfl(P[2], ib)};
    float ab[3];
    {
      const float amb[3] = {a[0] - b[0], a[1] - b[1], a[2] - b[2]};
      cross(ab, nr, amb);
    }
    const int ic = pick(fabsf((a[0] - P[0]) * ab[0] + (a[1] - P[1]) * ab[1] + (a[2] - P[2]) * ab[2]), mxv);
    const float cc[3] = {__shfl(P[0], ic), __shfl(P[1], ic), __shfl(P[2], ic)};
    float ac[3], bc[3];
    {
      const float amc[3] = {a[0] - cc[0], a[1] - cc[1], a[2] - cc[2]}, bmc[3] = {b[0] - cc[0], b[1] - cc[1], b[2] - cc[2]};
      cross(ac, nr, amc);
      cross(bc, nr, bmc);
    }
    float bbp, bap;
    const int ibp = pick(fabsf((b[0] - P[0]) * bc[0] + (b[1] - P[1]) * bc[1] + (b[2] - P[2]) * bc[2]), bbp);
    const int iap = pick(fabsf((a[0] - P[0]) * ac[0] + (a[1] - P[1]) * ac[1] + (a[2] - P[2]) * ac[2]), bap);
    idx[0] = ia; idx[1] = ib; idx[2] = ic; idx[3] = beats(bap, bbp) ? iap : ibp;
  }
#pragma unroll
  for (int j = 0; j < 4; j++) {
    bool dup = idx[j] < 0;
#pragma unroll
    for (int t = 0; t < j; t++) dup |= idx[t] == idx[j];
    const int L = idx[j] < 0 ? 0 : idx[j];
    const float Pj[3] = {__shfl(P[0], L), __shfl(P[1], L), __shfl(P[2], L)};
    const float dj = __shfl(dk, L);
    if (lane == q) {
      dist[j] = dup ? 1e30f : dj;
#pragma unroll
      for (int e = 0; e < 3; e++) { pos[j][e] = Pj[e] - 0.5f * dj * nr[e] + c[e]; nrm[j][e] = sg * nr[e]; }
    }
  }
  if (lane == q) nsl = 4;
  PSTAMP(m, 28);
}

// per-lane narrow phase for plane/capsule/box-vs-capsule pairs (box-box is
// wave-cooperative, below).  out: dist[4], pos[4][3], nrm[4][3]
template <class S>
__device__ __forceinline__ int narrow_lane(const DevModel* __restrict__ m, const S& s, short* hints, int p, float dist[4],
                            float pos[4][3], float nrm[4][3], float* dbg = nullptr) {
  const int g1 = m->pair_g1[p], g2 = m->pair_g2[p];
  const int func = m->pair_func[p];
  const float* x1 = s.gxpos[g1];
  const float* x2 = s.gxpos[g2];
  const float* R1 = s.gxmat[g1];
  const float* R2 = s.gxmat[g2];
  const float* s1 = m->geom_size[g1];
  const float* s2 = m->geom_size[g2];
#pragma unroll
  for (int k = 0; k < 4; k++) dist[k] = 1e30f;
  if (func == 0) {  // plane - capsule
    float n[3] = {R1[2], R1[5], R1[8]}, ax[3] = {R2[2], R2[5], R2[8]};
    float r = s2[0], hl = s2[1];
#pragma unroll
    for (int k = 0; k < 2; k++) {
      float sg = k == 0 ? 1.f : -1.f, e[3], dif[3];
#pragma unroll
      for (int c = 0; c < 3; c++) { e[c] = x2[c] + sg * hl * ax[c]; dif[c] = e[c] - x1[c]; }
      float d = dot3(n, dif) - r;
      dist[k] = d;
#pragma unroll
      for (int c = 0; c < 3; c++) { pos[k][c] = e[c] - n[c] * (r + 0.5f * d); nrm[k][c] = n[c]; }
    }
    return 2;
  }
  if (func == 1) {  // plane - box: the 4 deepest corners, ascending depth (ties: corner index)
    // depth(c) = n.(x2 - x1) + sum_k +-w_k with w_k = h_k n.R2_k: the deepest
    // corner takes the sign against each w_k, the next ones flip the axis of
    // the smallest |w|, of the second smallest, and then the third axis or
    // both of the first two -- 5 candidates instead of a 4 x 8 scan
    const float n[3] = {R1[2], R1[5], R1[8]};
    float w[3];
#pragma unroll
    for (int k = 0; k < 3; k++) w[k] = s2[k] * (n[0] * R2[k] + n[1] * R2[3 + k] + n[2] * R2[6 + k]);
    const int c0 = (w[0] < 0.f ? 1 : 0) | (w[1] < 0.f ? 2 : 0) | (w[2] < 0.f ? 4 : 0);
    int ax0 = 0, ax1 = 1, ax2 = 2;  // axes by |w| ascending, index order on ties
    if (fabsf(w[ax1]) < fabsf(w[ax0])) { const int t = ax0; ax0 = ax1; ax1 = t; }
    if (fabsf(w[ax2]) < fabsf(w[ax1])) { const int t = ax1; ax1 = ax2; ax2 = t; }
    if (fabsf(w[ax1]) < fabsf(w[ax0])) { const int t = ax0; ax0 = ax1; ax1 = t; }
    auto depth = [&](int c) {  // the same expression as the oracle's corner distance
      const float l[3] = {(c & 1) ? s2[0] : -s2[0], (c & 2) ? s2[1] : -s2[1], (c & 4) ? s2[2] : -s2[2]};
      float v[3];
      mv(v, R2, l);
      return n[0] * (x2[0] + v[0] - x1[0]) + n[1] * (x2[1] + v[1] - x1[1]) + n[2] * (x2[2] + v[2] - x1[2]);
    };
    int cs[4] = {c0, c0 ^ (1 << ax0), c0 ^ (1 << ax1), c0 ^ (1 << ax2)};
    float ds[4] = {depth(cs[0]), depth(cs[1]), depth(cs[2]), depth(cs[3])};
    {
      const int c4 = c0 ^ (1 << ax0) ^ (1 << ax1);
      const float d4 = depth(c4);
      if (d4 < ds[3] || (d4 == ds[3] && c4 < cs[3])) { cs[3] = c4; ds[3] = d4; }
    }
    // order the four by (depth, index): sorting network (0,1) (2,3) (0,2) (1,3) (1,2)
    auto cx = [&](int i, int j) {
      if (ds[j] < ds[i] || (ds[j] == ds[i] && cs[j] < cs[i])) {
        const float td = ds[i]; ds[i] = ds[j]; ds[j] = td;
        const int tc = cs[i]; cs[i] = cs[j]; cs[j] = tc;
      }
    };
    cx(0, 1); cx(2, 3); cx(0, 2); cx(1, 3); cx(1, 2);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int c = cs[k];
      const float l[3] = {(c & 1) ? s2[0] : -s2[0], (c & 2) ? s2[1] : -s2[1], (c & 4) ? s2[2] : -s2[2]};
      float v[3];
      mv(v, R2, l);
      dist[k] = ds[k];
#pragma unroll
      for (int e = 0; e < 3; e++) { pos[k][e] = x2[e] + v[e] - n[e] * 0.5f * ds[k]; nrm[k][e] = n[e]; }
    }
    return 4;
  }
  if (func == 2) {  // capsule - capsule
    float a1[3] = {R1[2], R1[5], R1[8]}, a2[3] = {R2[2], R2[5], R2[8]};
    float p1[3], d1[3], p2[3], d2[3];
#pragma unroll
    for (int c = 0; c < 3; c++) {
      p1[c] = x1[c] - s1[1] * a1[c]; d1[c] = 2 * s1[1] * a1[c];
      p2[c] = x2[c] - s2[1] * a2[c]; d2[c] = 2 * s2[1] * a2[c];
    }
    float sc, tc, n[3], c1[3];
    seg_seg(p1, d1, p2, d2, &sc, &tc);
#pragma unroll
    for (int c = 0; c < 3; c++) { c1[c] = p1[c] + sc * d1[c]; n[c] = p2[c] + tc * d2[c] - c1[c]; }
    float len = sqrtf(dot3(n, n));
    if (len < 1e-12f) {
      float t[3] = {1, 0, 0};
      if (fabsf(a1[0]) > 0.9f) { t[0] = 0; t[1] = 1; }
      cross(n, a1, t);
      float l = sqrtf(dot3(n, n));
      n[0] /= l; n[1] /= l; n[2] /= l;
    } else {
      n[0] /= len; n[1] /= len; n[2] /= len;
    }
    float d = len - s1[0] - s2[0];
    dist[0] = d;
#pragma unroll
    for (int c = 0; c < 3; c++) { pos[0][c] = c1[c] + n[c] * (s1[0] + 0.5f * d); nrm[0][c] = n[c]; }
    return 1;
  }
  if (func == 3) {  // capsule - box
    float ax[3] = {R1[2], R1[5], R1[8]}, r = s1[0], hl = s1[1];
    const float* h = s2;
    float A[3], B[3], a[3], dd[3];
#pragma unroll
    for (int c = 0; c < 3; c++) { A[c] = x1[c] - hl * ax[c] - x2[c]; B[c] = 2 * hl * ax[c]; }
    mtv(a, R2, A);
    mtv(dd, R2, B);
    float tlo = -1.f, thi = 2.f, flo = 0.f, fhi = 0.f;
    // knots: 0, 1, (+-h_k - a_k)/dd_k inside (0,1), where the squared
    // distance's derivative fp (piecewise linear, non-decreasing: the
    // distance is convex along the segment) is evaluated.  The interior knots
    // only matter when fp changes sign inside (fp(0) < 0 <= fp(1)); when no
    // lane's does, the minimum is an end on every lane (ts 0 or 1 below, as
    // the full scan gives) and the six interior knots are skipped (C3: most
    // steps of the 20 robot capsule / box pairs, MPCR_CB_SKIP)
    auto knot = [&](int i) {
      float t;
      bool ok = true;
      if (i == 0) t = 0.f;
      else if (i == 1) t = 1.f;
      else {
        int k = (i - 2) >> 1;
        float sg = ((i - 2) & 1) ? 1.f : -1.f;
        ok = fabsf(dd[k]) > kMinVal;
        t = ok ? (sg * h[k] - a[k]) / dd[k] : 0.f;
        ok = ok && t > 0.f && t < 1.f;
      }
      if (ok) {
        // x - clamp(x, -h, h) is +-(|x| - h) outside the slab, 0 inside --
        // the same value as the sign-selected excess, one v_med3 instead
        // of the compares and selects
        float fp = 0.f;
#pragma unroll
        for (int k = 0; k < 3; k++) {
          const float x = a[k] + t * dd[k];
          fp += 2.f * dd[k] * (x - __builtin_amdgcn_fmed3f(x, -h[k], h[k]));
        }
        if (fp < 0) { if (t > tlo) { tlo = t; flo = fp; } }
        else { if (t < thi) { thi = t; fhi = fp; } }
      }
    };
    knot(0);
    knot(1);
    if (!MPCR_CB_SKIP || hballot<S::CPW>(tlo == 0.f && thi == 1.f) != 0ull) {
#pragma unroll
      for (int i = 2; i < 8; i++) knot(i);
    }
    float ts;
    if (tlo < 0) ts = 0.f;
    else if (thi > 1) ts = 1.f;
    else ts = fhi - flo > 0 ? tlo - flo * (thi - tlo) / (fhi - flo) : tlo;
    float pp[3], q[3], nl[3];
#pragma unroll
    for (int c = 0; c < 3; c++) pp[c] = a[c] + ts * dd[c];
    float g = point_box(pp, h, nl, q);
    if (g <= 1e-6f && !MPCR_ABL_DEEP) {  // on or in the box (penetrating segments land on the surface): the oracle's band
      // deepest point of g(t) = max_k |x_k(t)| - h_k over its kinks
      float gbest = 1e30f, tbest = 0.f;
#pragma unroll
      for (int i = 0; i < 17; i++) {
        float t;
        bool ok = true;
        if (i == 0) t = 0.f;
        else if (i == 1) t = 1.f;
        else if (i < 5) {
          int k = i - 2;
          ok = fabsf(dd[k]) > kMinVal;
          t = ok ? -a[k] / dd[k] : 0.f;
          ok = ok && t > 0.f && t < 1.f;
        } else {
          int q4 = i - 5;        // 0..11: pair (ii,jj) x signs
          int pr = q4 >> 2;      // 0:(0,1) 1:(0,2) 2:(1,2)
          int ii = pr == 2 ? 1 : 0, jj = pr == 0 ? 1 : 2;
          float si = (q4 & 2) ? 1.f : -1.f, sj = (q4 & 1) ? 1.f : -1.f;
          float den = si * dd[ii] - sj * dd[jj];
          ok = fabsf(den) > kMinVal;
          t = ok ? (h[ii] - h[jj] - si * a[ii] + sj * a[jj]) / den : 0.f;
          ok = ok && t > 0.f && t < 1.f;
        }
        if (ok) {
          float gm = -1e30f;
#pragma unroll
          for (int k = 0; k < 3; k++) gm = fmaxf(gm, fabsf(a[k] + t * dd[k]) - h[k]);
          // a flat minimum (the segment parallel to a face: every kink as
          // deep) keeps the first candidate -- a later one must be deeper by
          // more than 1 um, so fp32 and fp64 pick the same point (the oracle's rule)
          if (gm < gbest - 1e-6f) { gbest = gm; tbest = t; }
        }
      }
      ts = tbest;
#pragma unroll
      for (int c = 0; c < 3; c++) pp[c] = a[c] + ts * dd[c];
      g = point_box(pp, h, nl, q);
    }
    // the far end: on or in the box, the first point's face, the segment
    // clipped to the face's extent (the oracle's col_capsule_box, round 4);
    // outside, its own point_box
    int fk = -1;
    float fsg = 0.f;
    if (g <= 0.f) {
#pragma unroll
      for (int c = 0; c < 3; c++)
        if (nl[c] != 0.f) { fk = c; fsg = -nl[c]; }
    }
#pragma unroll
    for (int k = 0; k < 2; k++) {
      if (k == 1) {
        float t = ts < 0.5f ? 1.f : 0.f;
        if (fk >= 0) {
#pragma unroll
          for (int j = 0; j < 3; j++) {
            if (j == fk || !(fabsf(dd[j]) > kMinVal)) continue;
            const float x = a[j] + t * dd[j];
            if (fabsf(x) > h[j]) {
              const float tb = ((x > 0.f ? h[j] : -h[j]) - a[j]) / dd[j];
              t = ts < t ? fminf(t, fmaxf(tb, ts)) : fmaxf(t, fminf(tb, ts));
            }
          }
          float gf = 0.f;
#pragma unroll
          for (int c = 0; c < 3; c++) {
            pp[c] = a[c] + t * dd[c];
            nl[c] = c == fk ? -fsg : 0.f;
            q[c] = c == fk ? fsg * h[c] : pp[c];
            gf = c == fk ? fsg * pp[c] - h[c] : gf;
          }
          g = gf;
        } else {
#pragma unroll
          for (int c = 0; c < 3; c++) pp[c] = a[c] + t * dd[c];
          g = point_box(pp, h, nl, q);
        }
      }
      float n[3], pl[3], tmp[3];
      mv(n, R2, nl);
#pragma unroll
      for (int c = 0; c < 3; c++) pl[c] = 0.5f * (pp[c] + r * nl[c] + q[c]);
      mv(tmp, R2, pl);
      dist[k] = g - r;
#pragma unroll
      for (int c = 0; c < 3; c++) { pos[k][c] = tmp[c] + x2[c]; nrm[k][c] = n[c]; }
    }
    return 2;
  }
  if constexpr (S::WIDE) {
    // hull hill climbs start where this pair's previous step ended (the
    // oracle keeps the same per-pair cache)
    int* hp = reinterpret_cast<int*>(hints) + (p - m->cvx_base);  // (side 0, side 1) as two shorts
    const int hv = *hp;
    int hint[2] = {(int)(short)(hv & 0xffff), hv >> 16};
    if (func == 9) {  // general convex (MPR)
      float depth, n[3], pp[3];
      float* tr = (dbg && (int)dbg[DBG_MPR] == p) ? dbg + DBG_MPR : nullptr;
      const bool hit = mpr_lane(m, s, g1, g2, depth, n, pp, hint, tr);
      if (tr) {
        tr[1] = hit ? 1.f : 0.f; tr[2] = depth;
        tr[3] = n[0]; tr[4] = n[1]; tr[5] = n[2]; tr[6] = pp[0]; tr[7] = pp[1]; tr[8] = pp[2];
      }
      *hp = (hint[0] & 0xffff) | (hint[1] << 16);
      if (hit) {
        if (n[0] == 0.f && n[1] == 0.f && n[2] == 0.f) n[2] = 1.f;
        dist[0] = -depth;
#pragma unroll
        for (int c = 0; c < 3; c++) { pos[0][c] = pp[c]; nrm[0][c] = n[c]; }
        // a penetrating polyhedron pair: the caller runs the face-clipping manifold
        if (m->pair_ncon[p] == 4 && depth > 0.f) return kPendingPoly;
      }
      return 1;
    }
    if (func == 10 && m->pair_ncon[p] == 4 && m->geom_type[g2] == 5) {
      // plane - cylinder: MuJoCo's mjc_PlaneCylinder (the oracle's
      // col_plane_cylinder): deepest rim point, the far cap's on that side,
      // two near-cap rim points 120 degrees either side of the first
      const float n[3] = {R1[2], R1[5], R1[8]};
      float ax[3] = {R2[2], R2[5], R2[8]}, vec[3];
      float prjaxis = dot3(n, ax);
      if (prjaxis > 0.f) { ax[0] = -ax[0]; ax[1] = -ax[1]; ax[2] = -ax[2]; prjaxis = -prjaxis; }
      const float dist0 = n[0] * (x2[0] - x1[0]) + n[1] * (x2[1] - x1[1]) + n[2] * (x2[2] - x1[2]);
#pragma unroll
      for (int c = 0; c < 3; c++) vec[c] = ax[c] * prjaxis - n[c];
      const float len = sqrtf(dot3(vec, vec));
      if (len < kMinVal) { vec[0] = R2[0]; vec[1] = R2[3]; vec[2] = R2[6]; }
      else { const float il = 1.f / len; vec[0] *= il; vec[1] *= il; vec[2] *= il; }
#pragma unroll
      for (int c = 0; c < 3; c++) { vec[c] *= s2[0]; ax[c] *= s2[1]; }
      const float prjvec = dot3(vec, n);
      prjaxis *= s2[1];
      const float margin = m->pair_margin[p];
      float d = dist0 + prjaxis + prjvec;
      dist[0] = d;
#pragma unroll
      for (int c = 0; c < 3; c++) { pos[0][c] = x2[c] + vec[c] + ax[c] - 0.5f * d * n[c]; nrm[0][c] = n[c]; }
      if (d <= margin) {
        d = dist0 - prjaxis + prjvec;
        if (d <= margin) {
          dist[1] = d;
#pragma unroll
          for (int c = 0; c < 3; c++) { pos[1][c] = x2[c] + vec[c] - ax[c] - 0.5f * d * n[c]; nrm[1][c] = n[c]; }
        }
        d = dist0 + prjaxis - 0.5f * prjvec;
        if (d <= margin) {
          float v1[3];
          cross(v1, vec, ax);
          const float l1 = sqrtf(dot3(v1, v1));
          const float sc = l1 > 0.f ? s2[0] * 0.8660254037844386f / l1 : 0.f;
#pragma unroll
          for (int k = 0; k < 2; k++) {
            const float sv = k ? -sc : sc;
            dist[2 + k] = d;
#pragma unroll
            for (int c = 0; c < 3; c++) {
              pos[2 + k][c] = x2[c] + sv * v1[c] + ax[c] - 0.5f * vec[c] - 0.5f * d * n[c];
              nrm[2 + k][c] = n[c];
            }
          }
        }
      }
      return 4;
    }
    if (func == 10) {  // plane - convex: deepest support point
      float n[3] = {R1[2], R1[5], R1[8]}, nn[3] = {-R1[2], -R1[5], -R1[8]}, q[3];
      support_geom(m, s, g2, nn, q, hint[1]);
      *hp = (hint[0] & 0xffff) | (hint[1] << 16);
      const float d = n[0] * (q[0] - x1[0]) + n[1] * (q[1] - x1[1]) + n[2] * (q[2] - x1[2]);
      dist[0] = d;
#pragma unroll
      for (int c = 0; c < 3; c++) { pos[0][c] = q[c] - 0.5f * d * n[c]; nrm[0][c] = n[c]; }
      // a penetrating mesh: the caller runs the wave-cooperative manifold
      return (d < 0.f && m->geom_type[g2] == 7) ? kPendingManifold : 1;
    }
  }
  return 0;
}

__device__ __forceinline__ void make_frame(float f[9], const float n[3]) {
  f[0] = n[0]; f[1] = n[1]; f[2] = n[2];
  float y[3] = {0.f, 1.f, 0.f};
  if (fabsf(n[1]) >= 0.5f) { y[1] = 0.f; y[2] = 1.f; }
  float dd = dot3(n, y);
  y[0] -= dd * n[0]; y[1] -= dd * n[1]; y[2] -= dd * n[2];
  float ny = sqrtf(dot3(y, y));
  f[3] = y[0] / ny; f[4] = y[1] / ny; f[5] = y[2] / ny;
  cross(f + 6, f, f + 3);
}

__device__ __forceinline__ float impedance(const float* si, float pos, float margin) {
  float dmin = clampf(si[0], kMinImp, kMaxImp), dmax = clampf(si[1], kMinImp, kMaxImp);
  float width = si[2], mid = si[3], power = si[4];
  if (dmin == dmax || width <= kMinVal) return 0.5f * (dmin + dmax);
  float x = fabsf((pos - margin) / width);
  if (x >= 1.f) return dmax;
  if (x <= 0.f) return dmin;
  float y;
  if (power == 1.f) y = x;
  else if (power == 2.f) y = x <= mid ? x * x / mid : 1.f - (1.f - x) * (1.f - x) / (1.f - mid);  // default solimp
  else if (x <= mid) y = powf(x, power) / powf(mid, power - 1.f);
  else y = 1.f - powf(1.f - x, power) / powf(1.f - mid, power - 1.f);
  return dmin + y * (dmax - dmin);
}

// Box-box, wave-cooperative (one pair, all 64 lanes, uniform control flow):
// lanes 0..14 evaluate the 15 separating axes, the reference-face clipping
// (Sutherland-Hodgman against the 4 side planes) runs with one lane per
// polygon edge and ballot compaction, the >4 selection is done on uniform
// values.  Same definitions and orders as the oracle's col_box_box.
// Appends up to 4 contacts to the active list.  Must be called by all lanes.
template <class S>
__device__ __forceinline__ void box_box_wave(const DevModel* __restrict__ m, S& s, int p, int lane) {
  const int g1 = m->pair_g1[p], g2 = m->pair_g2[p];
  const float margin = m->pair_margin[p];
  float x1[3], x2[3], axA[3][3], axB[3][3], t[3], ha[3], hb[3];
#pragma unroll
  for (int c = 0; c < 3; c++) {
    x1[c] = s.gxpos[g1][c];
    x2[c] = s.gxpos[g2][c];
    t[c] = x2[c] - x1[c];
    ha[c] = m->geom_size[g1][c];
    hb[c] = m->geom_size[g2][c];
  }
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int c = 0; c < 3; c++) { axA[i][c] = s.gxmat[g1][3 * c + i]; axB[i][c] = s.gxmat[g2][3 * c + i]; }
  // ---- separating axes, one per lane
  float L[3] = {0.f, 0.f, 1.f}, sep = -3e38f;
  bool valid = false;
  // (per-lane axes read from the LDS frames by index: no select chains)
  if (lane < 6) {
    const float* R = s.gxmat[lane < 3 ? g1 : g2];
    const int ia = lane < 3 ? lane : lane - 3;
#pragma unroll
    for (int c = 0; c < 3; c++) L[c] = R[3 * c + ia];
    valid = true;
  } else if (lane < 15) {
    const int i = (lane - 6) / 3, j = (lane - 6) % 3;
    float ai[3], bj[3];
#pragma unroll
    for (int c = 0; c < 3; c++) {
      ai[c] = s.gxmat[g1][3 * c + i];
      bj[c] = s.gxmat[g2][3 * c + j];
    }
    cross(L, ai, bj);
    const float l = sqrtf(dot3(L, L));
    valid = l >= 1e-6f;
    if (valid) { L[0] /= l; L[1] /= l; L[2] /= l; }
  }
  if (valid) {
    float ra = 0.f, rb = 0.f;
#pragma unroll
    for (int k = 0; k < 3; k++) { ra += ha[k] * fabsf(dot3(axA[k], L)); rb += hb[k] * fabsf(dot3(axB[k], L)); }
    sep = fabsf(dot3(t, L)) - ra - rb;
  }
  float best_face = -1e30f, best_edge = -1e30f;
  int face_id = -1, edge_lane = -1;
#pragma unroll
  for (int a = 0; a < 6; a++) {
    const float v = hrdlane<S::CPW>(sep, a);
    if (v > best_face) { best_face = v; face_id = a; }
  }
#pragma unroll
  for (int a = 6; a < 15; a++) {
    const float v = hrdlane<S::CPW>(sep, a);
    if (v > -1e30f && v > best_edge) { best_edge = v; edge_lane = a; }
  }
  const float best = fmaxf(best_face, best_edge);
  if (!(best < margin)) return;
  const bool use_edge = edge_lane >= 0 && best_edge > 0.95f * best_face + 1e-5f;
  const int src = use_edge ? edge_lane : face_id;
  float n[3] = {hrdlane<S::CPW>(L[0], src), hrdlane<S::CPW>(L[1], src), hrdlane<S::CPW>(L[2], src)};
  const float sg = dot3(t, n) >= 0.f ? 1.f : -1.f;
  n[0] *= sg; n[1] *= sg; n[2] *= sg;
  const int base = s.ncon;
  sync();
  if (use_edge) {
    const int ei = (edge_lane - 6) / 3, ej = (edge_lane - 6) % 3;
    float pa[3], pb[3], da[3], db[3];
#pragma unroll
    for (int c = 0; c < 3; c++) { pa[c] = x1[c]; pb[c] = x2[c]; }
#pragma unroll
    for (int k = 0; k < 3; k++) {
      if (k != ei) {
        const float s_ = dot3(n, axA[k]) >= 0.f ? 1.f : -1.f;
#pragma unroll
        for (int c = 0; c < 3; c++) pa[c] += s_ * ha[k] * axA[k][c];
      }
      if (k != ej) {
        const float s_ = dot3(n, axB[k]) >= 0.f ? -1.f : 1.f;
#pragma unroll
        for (int c = 0; c < 3; c++) pb[c] += s_ * hb[k] * axB[k][c];
      }
    }
    const float hae = m->geom_size[g1][ei], hbe = m->geom_size[g2][ej];
#pragma unroll
    for (int c = 0; c < 3; c++) {
      const float ae = s.gxmat[g1][3 * c + ei], be = s.gxmat[g2][3 * c + ej];
      pa[c] -= hae * ae; da[c] = 2.f * hae * ae;
      pb[c] -= hbe * be; db[c] = 2.f * hbe * be;
    }
    float sc, uc;
    seg_seg(pa, da, pb, db, &sc, &uc);
    if (lane == 0 && base < S::MAXACT) {
      float f[9];
      make_frame(f, n);
#pragma unroll
      for (int c = 0; c < 3; c++) s.con_pos[base][c] = 0.5f * (pa[c] + sc * da[c] + pb[c] + uc * db[c]);
#pragma unroll
      for (int e = 0; e < S::FRAMEW; e++) s.con_frame[base][e] = f[e];
      s.con_dist[base] = best_edge;
      s.con_pair[base] = p;
    }
    sync();
    if (lane == 0) s.ncon = base + 1;
    sync();
    return;
  }
  // ---- face contact: reference box owns the face axis.  The run-time axis
  // indices address the boxes' LDS frames and model sizes directly (no
  // select chains, nothing in scratch); same values as the registers above.
  const bool refA = face_id < 3;
  const int fi = refA ? face_id : face_id - 3;
  const int gr = refA ? g1 : g2, gn = refA ? g2 : g1;
  const float* Rr = s.gxmat[gr];  // axis k of a box: (R[k], R[3 + k], R[6 + k])
  const float* Ri = s.gxmat[gn];
  const float* hr = m->geom_size[gr];
  const float* hi = m->geom_size[gn];
  float cr[3], ci[3], nf[3];
#pragma unroll
  for (int c = 0; c < 3; c++) {
    cr[c] = s.gxpos[gr][c];
    ci[c] = s.gxpos[gn][c];
    nf[c] = refA ? n[c] : -n[c];
  }
  const float d0 = fabsf(Ri[0] * nf[0] + Ri[3] * nf[1] + Ri[6] * nf[2]);
  const float d1 = fabsf(Ri[1] * nf[0] + Ri[4] * nf[1] + Ri[7] * nf[2]);
  const float d2 = fabsf(Ri[2] * nf[0] + Ri[5] * nf[1] + Ri[8] * nf[2]);
  int ki = 0;
  float bestdot = d0;
  if (d1 > bestdot) { bestdot = d1; ki = 1; }
  if (d2 > bestdot) { bestdot = d2; ki = 2; }
  const int u = ki == 0 ? 1 : (ki == 1 ? 2 : 0), v = ki == 0 ? 2 : (ki == 1 ? 0 : 1);
  float Ik[3], Iu[3], Iv[3];
#pragma unroll
  for (int c = 0; c < 3; c++) {
    Ik[c] = Ri[3 * c + ki];
    Iu[c] = Ri[3 * c + u];
    Iv[c] = Ri[3 * c + v];
  }
  const float hk = hi[ki], hu = hi[u], hv = hi[v];
  const float si = dot3(Ik, nf) > 0.f ? -1.f : 1.f;
  if (lane < 4) {
    const float su = (lane == 0 || lane == 3) ? 1.f : -1.f, sv = lane < 2 ? 1.f : -1.f;
#pragma unroll
    for (int k = 0; k < 3; k++) s.poly[0][lane][k] = ci[k] + si * hk * Ik[k] + su * hu * Iu[k] + sv * hv * Iv[k];
  }
  int np = 4, cur = 0;
  // fast path: an incident face wholly inside the reference face's 4 side
  // planes (an object resting inside a table top) passes every clip unchanged
  // -- Sutherland-Hodgman keeps each vertex and adds no crossing -- so the 4
  // sequential clips are skipped for exactly the same polygon
  bool inside = true;
  sync();
  if (lane < 4) {
    const float P[3] = {s.poly[0][lane][0], s.poly[0][lane][1], s.poly[0][lane][2]};
#pragma unroll
    for (int pl = 0; pl < 4; pl++) {  // the clip loop's own dp expression
      const int ax = (fi + 1 + (pl >> 1)) % 3;
      const float sgn = (pl & 1) ? -1.f : 1.f;
      const float Ra[3] = {Rr[ax], Rr[3 + ax], Rr[6 + ax]};
      const float cra = dot3(cr, Ra);
      inside = inside && sgn * (dot3(P, Ra) - cra) - hr[ax] <= 0.f;
    }
  }
  if (hballot<S::CPW>(!inside) == 0ull) np = -np;  // marker: skip the clips
  for (int pl = 0; pl < 4 && np > 0; pl++) {
    sync();
    const int ax = (fi + 1 + (pl >> 1)) % 3;
    const float sgn = (pl & 1) ? -1.f : 1.f;
    const float Ra[3] = {Rr[ax], Rr[3 + ax], Rr[6 + ax]};
    const float hax = hr[ax];
    const float cra = dot3(cr, Ra);
    float P[3] = {0.f, 0.f, 0.f}, Q[3] = {0.f, 0.f, 0.f}, dp = 0.f, dq = 0.f;
    int e0 = 0, e1 = 0;
    if (lane < np) {
      const int c2 = lane + 1 == np ? 0 : lane + 1;
#pragma unroll
      for (int k = 0; k < 3; k++) { P[k] = s.poly[cur][lane][k]; Q[k] = s.poly[cur][c2][k]; }
      dp = sgn * (dot3(P, Ra) - cra) - hax;
      dq = sgn * (dot3(Q, Ra) - cra) - hax;
      e0 = dp <= 0.f;
      e1 = (dp < 0.f && dq > 0.f) || (dp > 0.f && dq < 0.f);
    }
    int tot;
    const int o = hscan_excl<S::CPW>(e0 + e1, tot);
    if (e0) {
#pragma unroll
      for (int k = 0; k < 3; k++) s.poly[cur ^ 1][o][k] = P[k];
    }
    if (e1) {
      const float wgt = dp / (dp - dq);
#pragma unroll
      for (int k = 0; k < 3; k++) s.poly[cur ^ 1][o + e0][k] = P[k] + wgt * (Q[k] - P[k]);
    }
    np = tot;
    cur ^= 1;
  }
  if (np < 0) np = -np;
  sync();
  if (np == 0) return;
  const float hrf = hr[fi];
  float depth = -3e38f;
  bool keep = false;
  if (lane < np) {
    const float rel[3] = {s.poly[cur][lane][0] - cr[0], s.poly[cur][lane][1] - cr[1], s.poly[cur][lane][2] - cr[2]};
    depth = hrf - dot3(rel, nf);
    keep = -depth < margin;
  }
  const unsigned long long km = hballot<S::CPW>(keep);
  const int nkeep = __popcll(km);
  if (nkeep == 0) return;
  const int rank = lanes_below(km);  // position of this lane among the kept points
  int slot = keep ? rank : -1;
  int npick = nkeep;
  if (nkeep > 4) {
    // deepest kept point (first maximum), then evenly spaced around the polygon
    int d0 = 0;
    float dbest = -3e38f;
#pragma unroll
    for (int c = 0; c < 8; c++) {
      const int cb = c + hbase<S::CPW>();  // lane c of this group
      const float dc = hrdlane<S::CPW>(depth, c);
      const bool kc = (km >> cb) & 1ull;
      const int rc = __popcll(km & ((1ull << cb) - 1ull));
      if (kc && dc > dbest) { dbest = dc; d0 = rc; }
    }
    slot = -1;
#pragma unroll
    for (int q = 0; q < 4; q++)
      if (keep && rank == (d0 + q * nkeep / 4) % nkeep) slot = q;
    npick = 4;
  }
  if (slot >= 0 && base + slot < S::MAXACT) {
    const int o = base + slot;
    float f[9];
    make_frame(f, n);
#pragma unroll
    for (int k = 0; k < 3; k++) s.con_pos[o][k] = s.poly[cur][lane][k] + nf[k] * 0.5f * depth;
#pragma unroll
    for (int e = 0; e < S::FRAMEW; e++) s.con_frame[o][e] = f[e];
    s.con_dist[o] = -depth;
    s.con_pair[o] = p;
  }
  sync();
  if (lane == 0) s.ncon = base + npick;
  sync();
}

// Per-lane contact bookkeeping after a narrow-phase pass: cost_c on the
// robot-masked slots (SBP/mjx_planner.py:284-296) and ballot-compacted append
// of the active contacts.  Must be called by all lanes (two barriers).
// Previous-step masked slot distances (cost_c's history term) of the lane's
// own pairs, held in registers across the horizon (narrow variant): the lane
// that owns pair p in 64-pair chunk k owns its <= 4 slots every step, so
// chunk k < NC keeps them in v[k][0..3] (no per-step HBM slab round trip: the
// slab's L2 evictions were ~8.6 MB of a C3 launch's 29.7 MB HBM traffic);
// pairs of later chunks use the slab.  The dual-arm class keeps the slab.
#ifndef MPCR_N_CPREV_REG
#define MPCR_N_CPREV_REG 1
#endif
template <class S>
struct SlotHist {
  static constexpr int NC = (!S::WIDE && MPCR_N_CPREV_REG) ? 128 / S::HL : 0;
  float v[NC > 0 ? NC : 1][4];
};

// the active contacts (dist < margin) of pair p into the contact list from
// position o on (those past MAXACT are dropped; the caller counts them)
template <class S>
__device__ __forceinline__ void put_contacts(const DevModel* __restrict__ m, S& s, int o, int p, int nsl,
                                             const float dist[4], const float pos[4][3], const float nrm[4][3]) {
  const float mg = m->pair_margin[p];
#pragma unroll
  for (int c = 0; c < 4; c++) {
    if (c < nsl && dist[c] < mg) {
      if (o < S::MAXACT) {
        float f[9];
        make_frame(f, nrm[c]);
        s.con_pos[o][0] = pos[c][0]; s.con_pos[o][1] = pos[c][1]; s.con_pos[o][2] = pos[c][2];
#pragma unroll
        for (int e = 0; e < S::FRAMEW; e++) s.con_frame[o][e] = f[e];
        s.con_dist[o] = dist[c];
        s.con_pair[o] = p;
      }
      o++;
    }
  }
}

template <class S>
__device__ __forceinline__ void emit_contacts(const DevModel* __restrict__ m, S& s, const RolloutArgs& args, int b,
                                              int t, int H, bool valid, int p, int nsl, const float dist[4],
                                              const float pos[4][3], const float nrm[4][3], float& cost_c,
                                              SlotHist<S>& sh, int k) {
  int act = 0;
  if (valid) {
    const int sa = m->pair_slotadr[p];
    if (sa >= 0) {
      const int ns = m->pair_ncon[p];
#pragma unroll
      for (int c = 0; c < 4; c++) {
        if (c < ns) {
          const float d = dist[c];
          if (d < 0.f) cost_c += 1.f;
          if (SlotHist<S>::NC > 0 && k < SlotHist<S>::NC) {  // this lane's registers (chunk k, slot c)
            float prev = 0.f;
#pragma unroll
            for (int j = 0; j < SlotHist<S>::NC; j++) prev = j == k ? sh.v[j][c] : prev;
            if (t > 0) cost_c += fmaxf(prev * (1.f - 0.005f) - d, 0.f);
#pragma unroll
            for (int j = 0; j < SlotHist<S>::NC; j++) sh.v[j][c] = j == k ? d : sh.v[j][c];
          } else {
            float* cp = S::CPREV_GLOBAL ? args.slot_prev + (size_t)b * m->nslot : s.cprev;
            if (t > 0) cost_c += fmaxf(cp[sa + c] * (1.f - 0.005f) - d, 0.f);
            cp[sa + c] = d;
          }
          if (args.trace_slots && b < args.n) args.trace_slots[((size_t)b * H + t) * m->nslot + sa + c] = d;
        }
      }
    }
    if (!(m->disableflags & 16)) {
      const float mg = m->pair_margin[p];
#pragma unroll
      for (int c = 0; c < 4; c++) act += (c < nsl && dist[c] < mg) ? 1 : 0;
    }
  }
  int tot;
  const int pre = hscan_excl<S::CPW>(act, tot);
  const int base = s.ncon;
  if (act) put_contacts(m, s, base + pre, p, nsl, dist, pos, nrm);
  sync();
  if (hlane<S::CPW>() == 0) s.ncon = base + tot;
  sync();
}

// ---------------------------------------------------------------------------
// line search point (MJX-style, see oracle)

// cost: complete, or (narrow kernel, full == false) without its constant
// part q0 (the active rows' 0.5 D jar^2 + the Gauss term), which the bracket
// never reads: the line search adds it once for the final two points.
// T: the precision of a point's step size, cost and derivatives and of the
// bracket arithmetic -- fp64 in the dual-arm class (LsReal): the point's cost
// alpha^2 q2 + alpha q1 + q0 cancels a ~1e4 constant to compare candidates
// that differ in the last fp32 bits, and the bracket's Newton steps
// alpha - d0 / d1 divide two such differences; in fp32 those decisions
// halved the dual arm's parity (78 -> 37 well-conditioned
// misses of the fp32 restatement against fp64).  The row sums stay fp32.
template <class T>
struct LsPtT { T alpha, cost, d0, d1; bool full; };
#ifndef MPCR_W_LS64
#define MPCR_W_LS64 1  // 0: the dual-arm line search in fp32 (timing experiments only)
#endif
template <class S>
using LsReal = typename std::conditional<S::WIDE && MPCR_W_LS64, double, float>::type;

// elliptic rows: efc_src = (5 << 24) | (contact << 14) | (pair << 4) | side
__device__ __forceinline__ bool ell_row(int src) { return (src >> 24) == 5; }
__device__ __forceinline__ bool ell_head(int src) { return (src >> 24) == 5 && (src & 15) == 0; }
__device__ __forceinline__ int ell_pair(int src) { return (src >> 4) & 1023; }


// the row's side of its kink at the step size alpha (in alpha's precision)
template <class T>
__device__ __forceinline__ bool ls_neg(float jar, float jv, T alpha) {
  return (T)jar + alpha * (T)jv < (T)0;
}

template <class S, class T>
__device__ __forceinline__ void ls_rows(const S& s, int lane, T alpha, float& q0, float& q1, float& q2) {
  q0 = q1 = q2 = 0.f;
  for (int r = lane; r < s.nefc; r += S::HL) {
    float jar = s.efc_jar[r], jv = s.efc_jv[r];
    if constexpr (S::WIDE) {
      if (ell_row(s.efc_src[r])) continue;
    }
    if (((s.efc_src[r] >> 24) == 1) || ls_neg(jar, jv, alpha)) {
      float D = s.efc_D[r];
      q0 += 0.5f * D * jar * jar;
      q1 += D * jv * jar;
      q2 += 0.5f * D * jv * jv;
    }
  }
}

template <class T>
__device__ __forceinline__ LsPtT<T> ls_make(T alpha, T q0, T q1, T q2) {
  LsPtT<T> p;
  p.alpha = alpha;
  p.cost = alpha * alpha * q2 + alpha * q1 + q0;
  p.d0 = (T)2 * alpha * q2 + q1;
  p.d1 = (T)2 * q2 + (q2 == (T)0 ? (T)kMinVal : (T)0);
  p.full = true;
  return p;
}

template <class S, bool Q0 = true, class T = LsReal<S>>
__device__ __forceinline__ LsPtT<T> ls_eval(const S& s, int lane, const float qg[3], T alpha) {
  float q0, q1, q2;
  ls_rows(s, lane, alpha, q0, q1, q2);
  q0 = Q0 ? hsum<S::CPW>(q0) + qg[0] : 0.f;
  q1 = hsum<S::CPW>(q1) + qg[1];
  q2 = hsum<S::CPW>(q2) + qg[2];
  LsPtT<T> p = ls_make<T>(alpha, q0, q1, q2);
  p.full = Q0;
  return p;
}
// the deferred constant parts of two line-search points in one row pass
template <class S, class T>
__device__ __forceinline__ void ls_finish(const S& s, int lane, const float qg[3], LsPtT<T>& a, LsPtT<T>& b) {
  float qa = 0.f, qb = 0.f;
  for (int r = lane; r < s.nefc; r += S::HL) {
    const float jar = s.efc_jar[r], jv = s.efc_jv[r];
    const bool eq = (s.efc_src[r] >> 24) == 1;
    const float c0 = 0.5f * s.efc_D[r] * jar * jar;
    if (eq || ls_neg(jar, jv, a.alpha)) qa += c0;
    if (eq || ls_neg(jar, jv, b.alpha)) qb += c0;
  }
  qa = hsum<S::CPW>(qa) + qg[0];
  qb = hsum<S::CPW>(qb) + qg[0];
  if (!a.full) { a.cost = a.cost + qa; a.full = true; }
  if (!b.full) { b.cost = b.cost + qb; b.full = true; }
}

// three line-search points in one pass over the rows; the 9 reductions are
// independent so their DPP chains interleave
template <class S, bool Q0 = true, class T = LsReal<S>>
__device__ __forceinline__ void ls_eval3(const S& s, int lane, const float qg[3], T a0, T a1, T a2,
                                         LsPtT<T>& p0, LsPtT<T>& p1, LsPtT<T>& p2) {
  float q[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const T al[3] = {a0, a1, a2};
  for (int r = lane; r < s.nefc; r += S::HL) {
    const float jar = s.efc_jar[r], jv = s.efc_jv[r], D = s.efc_D[r];
    const bool eq = (s.efc_src[r] >> 24) == 1;
    if constexpr (S::WIDE) {
      if (ell_row(s.efc_src[r])) continue;
    }
    const float c0 = 0.5f * D * jar * jar, c1 = D * jv * jar, c2 = 0.5f * D * jv * jv;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      if (eq || ls_neg(jar, jv, al[k])) { q[3 * k] += c0; q[3 * k + 1] += c1; q[3 * k + 2] += c2; }
    }
  }
#pragma unroll
  for (int k = 0; k < 9; k++) q[k] = (Q0 || k % 3) ? hsum<S::CPW>(q[k]) + qg[k % 3] : 0.f;
  p0 = ls_make<T>(a0, q[0], q[1], q[2]);
  p1 = ls_make<T>(a1, q[3], q[4], q[5]);
  p2 = ls_make<T>(a2, q[6], q[7], q[8]);
  p0.full = p1.full = p2.full = Q0;
}

// ---------------------------------------------------------------------------
// elliptic friction cone of one condim-3 contact (rows n, t1, t2; equal
// sliding frictions), MuJoCo's primal three-zone cost (oracle: ell_update /
// ell_line).  N = mu x_n, U = fri x_t, T = |U|:
//   top    N >= mu T        no cost
//   bottom mu N + T <= 0    0.5 sum D_k x_k^2
//   middle                  0.5 Dm (N - mu T)^2, Dm = D_n / (mu^2 (1 + mu^2))

// cost; f = -dcost/dx; h = Hessian (h00 h01 h02 h11 h12 h22)
__device__ __forceinline__ float cone_update(const float x[3], float mu, float fri, const float D[3], float f[3],
                                             float h[6]) {
  const float N = mu * x[0], U0 = fri * x[1], U1 = fri * x[2], T = sqrtf(U0 * U0 + U1 * U1);
  if (N >= mu * T || (T <= 0.f && N >= 0.f)) {
    f[0] = f[1] = f[2] = 0.f;
#pragma unroll
    for (int k = 0; k < 6; k++) h[k] = 0.f;
    return 0.f;
  }
  if (mu * N + T <= 0.f || (T <= 0.f && N < 0.f)) {
    f[0] = -D[0] * x[0]; f[1] = -D[1] * x[1]; f[2] = -D[2] * x[2];
    h[0] = D[0]; h[1] = 0.f; h[2] = 0.f; h[3] = D[1]; h[4] = 0.f; h[5] = D[2];
    return 0.5f * (D[0] * x[0] * x[0] + D[1] * x[1] * x[1] + D[2] * x[2] * x[2]);
  }
  const float Dm = D[0] / (mu * mu * (1.f + mu * mu)), phi = N - mu * T, iT = 1.f / T;
  const float g[3] = {mu, -mu * fri * U0 * iT, -mu * fri * U1 * iT};
  f[0] = -Dm * phi * g[0]; f[1] = -Dm * phi * g[1]; f[2] = -Dm * phi * g[2];
  const float c = -Dm * phi * mu * fri * fri * iT, u0 = U0 * iT, u1 = U1 * iT;
  h[0] = Dm * g[0] * g[0];
  h[1] = Dm * g[0] * g[1];
  h[2] = Dm * g[0] * g[2];
  h[3] = Dm * g[1] * g[1] + c * (1.f - u0 * u0);
  h[4] = Dm * g[1] * g[2] - c * u0 * u1;
  h[5] = Dm * g[2] * g[2] + c * (1.f - u1 * u1);
  return 0.5f * Dm * phi * phi;
}

// cost and its first two derivatives along x + alpha v (zones at alpha)
template <class A>
__device__ __forceinline__ void cone_line(const float x0[3], const float v[3], A alpha, float mu, float fri,
                                          const float D[3], float& c0, float& c1, float& c2) {
  const float x[3] = {(float)((A)x0[0] + alpha * (A)v[0]), (float)((A)x0[1] + alpha * (A)v[1]),
                      (float)((A)x0[2] + alpha * (A)v[2])};
  const float N = mu * x[0], U0 = fri * x[1], U1 = fri * x[2], W0 = fri * v[1], W1 = fri * v[2];
  const float T = sqrtf(U0 * U0 + U1 * U1);
  if (N >= mu * T || (T <= 0.f && N >= 0.f)) { c0 = c1 = c2 = 0.f; return; }
  if (mu * N + T <= 0.f || (T <= 0.f && N < 0.f)) {
    c0 = 0.5f * (D[0] * x[0] * x[0] + D[1] * x[1] * x[1] + D[2] * x[2] * x[2]);
    c1 = D[0] * x[0] * v[0] + D[1] * x[1] * v[1] + D[2] * x[2] * v[2];
    c2 = D[0] * v[0] * v[0] + D[1] * v[1] * v[1] + D[2] * v[2] * v[2];
    return;
  }
  const float Dm = D[0] / (mu * mu * (1.f + mu * mu));
  const float T1 = (U0 * W0 + U1 * W1) / T, T2 = (W0 * W0 + W1 * W1 - T1 * T1) / T;
  const float phi = N - mu * T, phi1 = mu * v[0] - mu * T1, phi2 = -mu * T2;
  c0 = 0.5f * Dm * phi * phi;
  c1 = Dm * phi * phi1;
  c2 = Dm * (phi1 * phi1 + phi * phi2);
}

template <class S>
__device__ __forceinline__ const float* jrow_ptr(const S& s, const float* gx, int r) {
  return (S::JL == S::MAXEFC || r < S::JL) ? &s.J[r][0] : gx + (r - S::JL) * S::LDJ;
}

// line-search extra terms of the elliptic contacts at three step sizes
template <class S, class T>
__device__ __forceinline__ void ls_cones3(const S& s, const DevModel* __restrict__ m, int lane, const T al[3],
                                          float e[9]) {
#pragma unroll
  for (int k = 0; k < 9; k++) e[k] = 0.f;
  for (int r = lane; r < s.nefc; r += S::HL) {
    const int src = s.efc_src[r];
    if (!ell_head(src)) continue;
    const int p = ell_pair(src);
    const float x[3] = {s.efc_jar[r], s.efc_jar[r + 1], s.efc_jar[r + 2]};
    const float v[3] = {s.efc_jv[r], s.efc_jv[r + 1], s.efc_jv[r + 2]};
    const float D[3] = {s.efc_D[r], s.efc_D[r + 1], s.efc_D[r + 2]};
#pragma unroll
    for (int k = 0; k < 3; k++) {
      float c0, c1, c2;
      cone_line(x, v, al[k], m->pair_cmu[p], m->pair_friction[p], D, c0, c1, c2);
      e[3 * k] += c0; e[3 * k + 1] += c1; e[3 * k + 2] += c2;
    }
  }
#pragma unroll
  for (int k = 0; k < 9; k++) e[k] = hsum<S::CPW>(e[k]);
}

template <class T>
__device__ __forceinline__ void ls_add(LsPtT<T>& p, float c0, float c1, float c2) {
  p.cost += (T)c0;
  p.d0 += (T)c1;
  p.d1 = p.d1 - (p.d1 == (T)kMinVal ? (T)kMinVal : (T)0) + (T)c2;
  if (p.d1 == (T)0) p.d1 = (T)kMinVal;
}

// Re-derive the model pointer from the kernel argument through an opaque
// zero offset.  The compiler then cannot hoist loop-invariant model loads out
// of the horizon loop (which kept them all live: 244 VGPRs), while the base
// stays a kernel-argument pointer so its loads remain global (uniform ones
// scalar) instead of FLAT.
#define LAUNDER_MODEL()                  \
  do {                                   \
    int z_ = 0;                          \
    asm volatile("" : "+s"(z_));         \
    m = m0 + z_;                         \
  } while (0)
// The lane index is laundered once per step the same way (narrow variant):
// otherwise every lane-mask compare (lane > k in the register Cholesky,
// lane < nv, ...) is a loop invariant the compiler hoists out of the horizon
// loop into an SGPR pair, which then spills to VGPR lanes (two v_readlane per
// use) and keeps lane-derived addresses live across the step: 178 -> 130
// VGPRs, i.e. 3 waves/SIMD instead of 2 once the LDS image fits (below).
#ifndef MPCR_LANE_LAUNDER
#define MPCR_LANE_LAUNDER 1
#endif
#define LAUNDER_LANE() asm volatile("" : "+v"(lane))
#ifndef MPCR_W_LANE_LAUNDER
#define MPCR_W_LANE_LAUNDER 1  // the dual-arm kernel too: 256 -> 241 VGPRs, scratch 304 -> 144 B, C4 49.7 -> 48.6 ms
#endif
// phase-boundary launders (-DMPCR_PHASE_LAUNDER=0 keeps only the per-step one)
#ifndef MPCR_PHASE_LAUNDER
#define MPCR_PHASE_LAUNDER 0
#endif
#if MPCR_PHASE_LAUNDER
#define LAUNDER_PHASE() LAUNDER_MODEL()
#elif MPCR_LANE_LAUNDER >= 2 || MPCR_W_LANE_LAUNDER >= 2
#define LAUNDER_PHASE()                                                          \
  do {                                                                           \
    if constexpr (WIDE ? MPCR_W_LANE_LAUNDER >= 2 : MPCR_LANE_LAUNDER >= 2) LAUNDER_LANE(); \
  } while (0)
#else
#define LAUNDER_PHASE() \
  do {                  \
  } while (0)
#endif

// ---------------------------------------------------------------------------
// J row access: rows < JL in LDS, the rest in the block's HBM slab gx.  The
// branches are per lane, and the HBM side is skipped (execz) unless a lane
// has a row past JL.

template <class S>
__device__ __forceinline__ void jstore(S& s, float* gx, int r, int i, float v) {
  if (S::JL == S::MAXEFC || r < S::JL) s.J[r][i] = v;
  else gx[(r - S::JL) * S::LDJ + i] = v;
}
template <class S>
__device__ __forceinline__ float jdot(const S& s, const float* gx, int r, const float* vec) {
  if (S::JL == S::MAXEFC || r < S::JL) return dotN<S::NVW>(s.J[r], vec);
  return dotN<S::NVW>(gx + (r - S::JL) * S::LDJ, vec);
}
// body(row pointer, r) over rows r = r0, r0 + step, ... < nefc: the LDS rows,
// then the slab rows (two loops, no per-row address-space select)
template <class S, class F>
__device__ __forceinline__ void jrows(const S& s, const float* gx, int r0, int step, int nefc, F&& body) {
  const int n1 = nefc < S::JL ? nefc : S::JL;
  for (int r = r0; r < n1; r += step) body(&s.J[r][0], r);
  if constexpr (S::JL < S::MAXEFC) {
    for (int r = S::JL + r0; r < nefc; r += step) body(gx + (r - S::JL) * S::LDJ, r);
  }
}

// ---------------------------------------------------------------------------
// the kernel

// The narrow variant is compiled for 4 waves/SIMD (<= 128 VGPRs; its LDS image
// fits 16 blocks per CU): at the bench's 4096 candidates = 4 per SIMD every
// candidate is resident at once (3 waves/SIMD: 3.52 ms, 4: 2.76 ms on C3).
#ifndef MPCR_DPP_CHOL
#define MPCR_DPP_CHOL 1
#endif
// narrow variant: the Newton gradient J^T f and Hessian J^T D J on the matrix
// core (v_mfma_f32_16x16x4_f32) instead of per-row VALU loops
#ifndef MPCR_MFMA_HESS
#define MPCR_MFMA_HESS 1
#endif
typedef float mfx4 __attribute__((ext_vector_type(4)));
typedef float mfx16 __attribute__((ext_vector_type(16)));
// narrow variant: the chain / subtree sums of the dynamics (CRB, body
// velocities, cdof_dot, RNE accelerations, bias forces) and the mass matrix as
// 16 x 16 (x 16) products on the matrix core: a 0/1 (or qvel-weighted) chain
// mask times per-dof / per-body rows.  v_mfma_f32_16x16x4_f32 is a k-ordered
// fmaf chain, and the products are the loops' own (qvel x cdof, fvec x cdof),
// so the results are bitwise the per-lane loops'
#ifndef MPCR_MFMA_DYN
#define MPCR_MFMA_DYN 1
#endif
// acc + A B over k < 16 (4 instructions): lane l supplies A[l & 15][k] =
// af(l & 15, k) and B[k][l & 15] = bf(k, l & 15) for its k = 4 s + (l >> 4);
// register v of lane l then holds row 4 (l >> 4) + v, column l & 15
template <int KB, class AF, class BF>
__device__ __forceinline__ mfx4 mm16(AF&& af, BF&& bf, mfx4 acc, int lane) {
  const int i = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int s4 = 0; s4 < KB; s4++) {
    const int k = 4 * s4 + kq;
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(af(i, k), bf(k, i), acc, 0, 0, 0);
  }
  return acc;
}
// the same for the 32-wide (dual-arm) Newton on v_mfma_f32_32x32x2_f32
// (neutral while the 32-wide readlane Cholesky dominated; with the blocked
// per-tree solve C4 66.2 -> 65.2 ms)
#ifndef MPCR_MFMA_HESS_W
#define MPCR_MFMA_HESS_W 1
#endif
// two waves per candidate, dual-arm class: wave 1 builds each Newton
// iteration's Hessian while wave 0 forms J^T f, the gradient and the stop test
#ifndef MPCR_W2_HESS
#define MPCR_W2_HESS 1
#endif
// ... and the implicit solve's blocked factor of M + dt D on wave 1 during Newton
#ifndef MPCR_W2_IMPL
#define MPCR_W2_IMPL 1
#endif
// The dual-arm variant is compiled for 2 waves/SIMD (<= 256 registers incl.
// AGPRs; uncapped it took 274 and ran 1 wave/SIMD): with its 21.6 KB image,
// 7 blocks per CU instead of 4 (dual arm 4096 x 50: 47.5 -> 35.8 ms).
#ifndef MPCR_W_WAVES
#define MPCR_W_WAVES 2
#endif
#ifndef MPCR_N_WAVES
#define MPCR_N_WAVES 4
#endif
// occupancy experiments: -DMPCR_WAVES_PER_EU=n asks the compiler for n waves/SIMD
#ifdef MPCR_WAVES_PER_EU
#define MPCR_ROLLOUT_ATTR __attribute__((amdgpu_waves_per_eu(MPCR_WAVES_PER_EU, MPCR_WAVES_PER_EU)))
#else
#define MPCR_ROLLOUT_ATTR
#endif

// 32-wide: acc += sum over constraint rows, two per v_mfma_f32_32x32x2_f32
// (lane (gi, gq) supplies A = J[r0 + gq][gi] and B = bf(r, A)).  Rows < JL
// come from LDS; the HBM-slab rows (heavily constrained candidates: 100+
// rows) are read four row pairs at a time with the loads issued together,
// instead of one dependent flat load per instruction.  Same MFMAs in the same
// row order (pairs wholly past nefc skipped): bitwise the single loop.
template <class S, class BF>
__device__ __forceinline__ mfx16 mfma_rows32(const S& s, const float* gx, int nefc, int gi, int gq, BF&& bf,
                                             mfx16 acc) {
  static_assert(S::JL % (MPCR_W_MFMA_SPLIT ? 8 : 2) == 0, "a row group never straddles the LDS / slab boundary");
#if MPCR_W_MFMA_SPLIT
  // two accumulators (row groups alternate), four row pairs' operands loaded
  // before their MFMAs: the dependent 32x32x2 chain and the LDS / slab loads
  // feeding it overlap (the sum is reassociated once at the end)
  mfx16 acc2;
#pragma unroll
  for (int v = 0; v < 16; v++) acc2[v] = 0.f;
  for (int r0 = 0; r0 < nefc; r0 += 8) {
    float a[4], bv[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int r = r0 + 2 * u + gq;
      a[u] = r < nefc ? (r < S::JL ? s.J[r][gi] : gx[(r - S::JL) * S::LDJ + gi]) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int r = r0 + 2 * u + gq;
      bv[u] = r < nefc ? bf(r, a[u]) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; u += 2) {
      if (r0 + 2 * u < nefc) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u], bv[u], acc, 0, 0, 0);
      if (r0 + 2 * u + 2 < nefc) acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u + 1], bv[u + 1], acc2, 0, 0, 0);
    }
  }
#pragma unroll
  for (int v = 0; v < 16; v++) acc[v] += acc2[v];
#else
  const int n1 = nefc < S::JL ? nefc : S::JL;
  for (int r0 = 0; r0 < n1; r0 += 2) {
    const int r = r0 + gq;
    const bool ok = r < nefc;
    const float a = ok ? s.J[r][gi] : 0.f;
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, ok ? bf(r, a) : 0.f, acc, 0, 0, 0);
  }
  if constexpr (S::JL < S::MAXEFC) {
    for (int r0 = S::JL; r0 < nefc; r0 += 8) {
      float a[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int r = r0 + 2 * u + gq;
        a[u] = r < nefc ? gx[(r - S::JL) * S::LDJ + gi] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int r = r0 + 2 * u + gq;
        if (r0 + 2 * u < nefc)
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u], r < nefc ? bf(r, a[u]) : 0.f, acc, 0, 0, 0);
      }
    }
  }
#endif
  return acc;
}

// WPC = waves per candidate.  WPC = 2 (narrow variant, small batches: one
// candidate per SIMD or fewer): wave 1 runs the collision
// phase while wave 0 runs the dynamics (cinert .. M^-1 qfrc_smooth) -- the two
// are independent given the step's kinematics -- and meets wave 0 at two
// workgroup barriers per step (geom poses ready; contacts ready).  Same
// instructions on the same data as WPC = 1, so the results are bitwise equal.
template <int NVW, int NBW, int NGW, bool WIDE, int WPC = 1>
__global__ void __launch_bounds__(WAVE * WPC, WIDE ? MPCR_W_WAVES : MPCR_N_WAVES / SmemN::CPW) MPCR_ROLLOUT_ATTR rollout_kernel(RolloutArgs args,
                                                                        const DevModel* __restrict__ mptr) {
  static_assert(WPC == 1 || (WPC == 2 && (WIDE || SmemN::CPW == 1)), "two waves per candidate: CPW 1");
  using S = typename std::conditional<WIDE, typename std::conditional<WPC == 2, SmemW2, SmemW>::type,
                                      typename std::conditional<WPC == 2, SmemN2, SmemN>::type>::type;
  const int wv = WPC == 2 ? (int)(threadIdx.x >> 6) : 0;
  const bool run_main = WPC == 1 || wv == 0, run_coll = WPC == 1 || wv == 1;
  static_assert(S::NVW == NVW && S::NBW == NBW && S::NGW == NGW, "variant widths");
  __shared__ S sm[S::CPW];  // one LDS image per candidate of the wave
  S& s = sm[S::CPW == 1 ? 0 : (int)(threadIdx.x >> 5)];
  const DevModel* __restrict__ const m0 = mptr;
  const DevModel* __restrict__ m = m0;
  int lane = hlane<S::CPW>();  // lane within the candidate's group; laundered per step (LAUNDER_LANE)
  const int b = blockIdx.x * S::CPW + (S::CPW == 1 ? 0 : (int)(threadIdx.x >> 5));
  const bool live = b < args.n;  // the last wave's second group may be empty
  if (S::CPW == 1 && !live) return;
  const int bi = live ? b : args.n - 1;  // an empty group replays a real candidate, writes nothing
  const int H = args.H;
  // horizon segment of this launch (dual-arm one-wave variant only)
  constexpr bool SEG = WIDE && WPC == 1 && S::CPW == 1;
  const int t_begin = SEG ? args.t0 : 0, t_end = SEG ? args.t1 : H;
  const bool resume = SEG && t_begin > 0, suspend = SEG && t_end < H;
  float* const segs = SEG ? args.seg_state + (size_t)b * SEG_STRIDE : nullptr;
  const int nv = m->nv, nb = m->nbody, nc = m->nctrl;
  float* const gx = S::JL < S::MAXEFC ? args.jx + (size_t)b * (S::MAXEFC - S::JL) * S::LDJ : nullptr;
  short* const hx = S::WIDE ? args.hints + (size_t)b * S::NHINT * 2 : nullptr;
  // mass matrix: the dense LDS image (single-arm variants), the compact LDS
  // rows of the dual-arm class (DevModel::mc_row: row i holds its tree's
  // columns; the others are 0 and rows past nv the identity), or -- a
  // dual-arm-class model whose compact M does not fit -- the candidate's HBM slab
  float* const mrow0 = S::M_SLAB ? args.mslab + (size_t)b * NVW * S::LD : nullptr;
  const bool mcomp = S::M_SLAB && m->mc_n > 0;
  constexpr int MCW = S::MCW;
  auto m_get = [&](int i, int j) -> float {
    if constexpr (S::M_SLAB) {
      if (mcomp) {
        if (i >= nv) return i == j ? 1.f : 0.f;
        const unsigned c = (unsigned)(j - m->mc_c0[i]);
        return c < (unsigned)MCW ? s.Mc[i * MCW + c] : 0.f;
      }
      return mrow0[i * S::LD + j];
    } else {
      return s.M[i][j];
    }
  };
  auto m_set = [&](int i, int j, float v) {
    if constexpr (S::M_SLAB) {
      if (mcomp) {
        const unsigned c = (unsigned)(j - m->mc_c0[i]);
        if (i < nv && c < (unsigned)MCW) s.Mc[i * MCW + c] = v;
        return;
      }
      mrow0[i * S::LD + j] = v;
    } else {
      s.M[i][j] = v;
    }
  };
  // the window start of this lane's row (lane mod NVW), read once: the row
  // accessors below run in the Newton loop, where a dependent model load in
  // front of every LDS read cost more than the HBM slab's L2 reads had
  const int mc0_lane = S::M_SLAB ? m->mc_c0[lane & (NVW - 1)] : 0;
  // columns 4q .. 4q + 3 of row i = this lane's row (lane mod NVW)
  auto m_quad = [&](int i, int q) -> float4 {
    if constexpr (S::M_SLAB) {
      if (mcomp) {
        if (i >= nv) {
          const int k = i - 4 * q;
          return make_float4(k == 0 ? 1.f : 0.f, k == 1 ? 1.f : 0.f, k == 2 ? 1.f : 0.f, k == 3 ? 1.f : 0.f);
        }
        const unsigned c = (unsigned)(4 * q - mc0_lane);
        const float4 v = *reinterpret_cast<const float4*>(&s.Mc[i * MCW + (c & (MCW - 4))]);
        return c < (unsigned)MCW ? v : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      return reinterpret_cast<const float4*>(mrow0 + i * S::LD)[q];
    } else {
      return reinterpret_cast<const float4*>(s.M[i])[q];
    }
  };
  // (M vec)[i], i = this lane's row, < nv: dotN's fmaf chain; a compact row
  // leaves out columns that are 0 (other trees') before and after its window,
  // which leaves the sum bitwise unchanged
  auto m_dot = [&](int i, const float* vec) -> float {
    if constexpr (S::M_SLAB) {
      if (mcomp) return dotN<MCW>(&s.Mc[i * MCW], vec + mc0_lane);
      return dotN<NVW>(mrow0 + i * S::LD, vec);
    } else {
      return dotN<NVW>(s.M[i], vec);
    }
  };
  // Newton Hessian H = M + J^T D_active J (+ the cone blocks) into Hs: lane
  // (row i, column quads q, q + RPW, ...) builds QPL float4s of row i, written
  // as LDS rows.  Wave 0's Newton step, or -- two waves, dual-arm class --
  // wave 1's, while wave 0 forms J^T f, the gradient and the stop test.
  auto newton_hessian = [&](int nefc, float* Hs) {
    constexpr bool MFMA_HESS_W = NVW == 32 && S::CPW == 1 && MPCR_MFMA_HESS_W;
    constexpr int RPW = S::HL / NVW;
    constexpr int QPL = NVW / 4 / RPW;
    const int gi = lane & (NVW - 1), gq = lane >> S::LOG_NVW;
    float4 hq[QPL];
#pragma unroll
    for (int k = 0; k < QPL; k++) hq[k] = m_quad(gi, gq + RPW * k);
    if constexpr (MFMA_HESS_W) {
      // J^T D J on v_mfma_f32_32x32x2_f32: accumulator register 4k + e of
      // lane (gi, gq) is H[gi][4 (gq + 2k) + e] in the transposed view --
      // exactly hq[k].e, the VALU build's ownership, and the same products
      // in the same row order (bitwise the VALU H)
      mfx16 acc;
#pragma unroll
      for (int k = 0; k < QPL; k++) {
        acc[4 * k] = hq[k].x; acc[4 * k + 1] = hq[k].y; acc[4 * k + 2] = hq[k].z; acc[4 * k + 3] = hq[k].w;
      }
      acc = mfma_rows32(s, gx, nefc, gi, gq, [&](int r, float a) { return s.efc_Da[r] * a; }, acc);
#pragma unroll
      for (int k = 0; k < QPL; k++) hq[k] = make_float4(acc[4 * k], acc[4 * k + 1], acc[4 * k + 2], acc[4 * k + 3]);
    } else {
      jrows(s, gx, 0, 1, nefc, [&](const float* J, int r) {
        const float c = s.efc_Da[r] * J[gi];
#pragma unroll
        for (int k = 0; k < QPL; k++) {
          const float4 v = reinterpret_cast<const float4*>(J)[gq + RPW * k];
          hq[k].x = fmaf(c, v.x, hq[k].x); hq[k].y = fmaf(c, v.y, hq[k].y);
          hq[k].z = fmaf(c, v.z, hq[k].z); hq[k].w = fmaf(c, v.w, hq[k].w);
        }
      });
    }
    if constexpr (S::WIDE) {  // cone Hessian blocks J_c^T H_c J_c (wave-uniform loop)
      if (m->cone == 1)
        for (int r = 0; r < nefc; r++) {
          const int src = s.efc_src[r];
          if (!ell_head(src)) continue;
          const int p = ell_pair(src);
          const float x[3] = {s.efc_jar[r], s.efc_jar[r + 1], s.efc_jar[r + 2]};
          const float D[3] = {s.efc_D[r], s.efc_D[r + 1], s.efc_D[r + 2]};
          float f[3], h[6];
          cone_update(x, m->pair_cmu[p], m->pair_friction[p], D, f, h);
          const float* J0 = jrow_ptr(s, gx, r);
          const float* J1 = jrow_ptr(s, gx, r + 1);
          const float* J2 = jrow_ptr(s, gx, r + 2);
          const float j0 = J0[gi], j1 = J1[gi], j2 = J2[gi];
          const float c0 = h[0] * j0 + h[1] * j1 + h[2] * j2;
          const float c1 = h[1] * j0 + h[3] * j1 + h[4] * j2;
          const float c2 = h[2] * j0 + h[4] * j1 + h[5] * j2;
#pragma unroll
          for (int k = 0; k < QPL; k++) {
            const float4 v0 = reinterpret_cast<const float4*>(J0)[gq + RPW * k];
            const float4 v1 = reinterpret_cast<const float4*>(J1)[gq + RPW * k];
            const float4 v2 = reinterpret_cast<const float4*>(J2)[gq + RPW * k];
            hq[k].x += c0 * v0.x + c1 * v1.x + c2 * v2.x;
            hq[k].y += c0 * v0.y + c1 * v1.y + c2 * v2.y;
            hq[k].z += c0 * v0.z + c1 * v1.z + c2 * v2.z;
            hq[k].w += c0 * v0.w + c1 * v1.w + c2 * v2.w;
          }
        }
    }
#pragma unroll
    for (int k = 0; k < QPL; k++) reinterpret_cast<float4*>(Hs + gi * S::LD)[gq + RPW * k] = hq[k];
    sync();
  };

  // ---- rollout init: template state, qpos[:nctrl] = init_pos ----------------
  //      (plant mode: the caller's state, no init_pos override)
  const bool from_state = (args.plant & 1) != 0;
  if (run_main) {  // (WPC = 2: wave 0 sets the image up, wave 1 waits at the barrier below)
  if (lane < PAR_N) s.par[lane] = args.dpar ? args.dpar[lane] : args.par[lane];
  if constexpr (S::SPLIT)
    if (lane == 0) s.ctok_[0] = 0;  // no step's pair cull posted yet
  if constexpr (S::WIDE) {
    // a rollout starts its hull climbs afresh; the plant keeps them across
    // steps (reset by mpcr_plant_set_state), so k plant steps = a k-step rollout
    if (!from_state && !resume) {
      int* h = reinterpret_cast<int*>(args.hints + (size_t)b * S::NHINT * 2);
      for (int i = lane; i < S::NHINT; i += S::HL) h[i] = -1;  // both sides -1
    }
  }
  if (resume) {  // a later horizon segment: the state the previous one saved
    for (int i = lane; i < S::NQW; i += S::HL) s.qpos[i] = i < DX_NQ ? segs[SEG_QPOS + i] : 0.f;
    if (lane < NVW) {
      s.qvel[lane] = segs[SEG_QVEL + lane];
      s.qws[lane] = segs[SEG_QWS + lane];
      s.qacc[lane] = 0.f;
    }
  } else {
  for (int i = lane; i < S::NQW; i += S::HL)
    s.qpos[i] = i < m->nq ? (from_state ? args.state[ST_QPOS + i] : m->qpos_init[i]) : 0.f;
  if (lane < NVW) {
    const bool v = lane < nv;
    s.qvel[lane] = v ? (from_state ? args.state[ST_QVEL + lane] : m->qvel_init[lane]) : 0.f;
    s.qws[lane] = v && from_state ? args.state[ST_QWS + lane] : 0.f;
    s.qacc[lane] = 0.f;
  }
  }
  sync();
  if (lane == 0) {  // normalise the target quaternion once
    const float* q = &s.par[PAR_QT];
    const float qn = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    s.par[PAR_QT] = q[0] / qn; s.par[PAR_QT + 1] = q[1] / qn; s.par[PAR_QT + 2] = q[2] / qn;
    s.par[PAR_QT + 3] = q[3] / qn;
  }
  if (lane < nc && !from_state && !resume) s.qpos[m->ctrl_qposadr[lane]] = s.par[PAR_Q0 + lane];
  sync();
  }
  if constexpr (WPC == 2) block_sync();

#if MPCR_TD_TABLE
  // the candidate's joint velocities for the whole horizon, computed up front
  // by all lanes (theta_dot = A_thetadot xi, SBP/mjx_planner.py:348) into the
  // thetadot output (or a scratch row); each step then reads its value with a
  // load issued one step ahead, so no per-step basis latency is exposed
  const float* tdp;
  if (args.layout == 0) {
    float* tdw = (args.thetadot && live ? args.thetadot : args.tdscratch) + (size_t)b * nc * H;
    for (int idx = lane; run_main && !resume && idx < nc * H; idx += S::HL) {
      const int j = idx / H, tt = idx - j * H;
      const float* pd = args.pdot + (size_t)tt * args.nbasis;
      const float* xj = args.input + ((size_t)bi * nc + j) * args.nbasis;
      float v = 0.f;
#pragma unroll
      for (int k = 0; k < 12; k++)
        if (k < args.nbasis) v = fmaf(pd[k], xj[k], v);
      tdw[idx] = v;
    }
    __threadfence_block();
    sync();
    if constexpr (WPC == 2) block_sync();
    tdp = tdw;
  } else {
    tdp = args.input + (size_t)bi * nc * H;
  }
  float vnext = lane < nc ? tdp[lane * H + t_begin] : 0.f;
#else
  // lane j < nctrl keeps joint j's Bernstein coefficients in registers for
  // the whole horizon (nbasis <= 12, checked by the engine)
  float xir[12];
#pragma unroll
  for (int k = 0; k < 12; k++)
    xir[k] = (args.layout == 0 && lane < nc && k < args.nbasis)
                 ? args.input[((size_t)bi * nc + lane) * args.nbasis + k] : 0.f;
#endif
  float cost_g = 0.f, cost_r = 0.f, cost_c = 0.f;
  SlotHist<S> shist;
#pragma unroll
  for (int j = 0; j < SlotHist<S>::NC; j++)
#pragma unroll
    for (int c = 0; c < 4; c++) shist.v[j][c] = 0.f;
  int status = 0, nefc_sum = 0, nefc_max = 0;
  if (resume) {  // the accumulators as the previous segment left them (lane 0's scalars on every lane)
    cost_c = segs[SEG_COSTC + lane];
    const float* sc = segs + SEG_SCAL;
    cost_g = sc[0]; cost_r = sc[1];
    status = __float_as_int(sc[2]); nefc_sum = __float_as_int(sc[3]); nefc_max = __float_as_int(sc[4]);
  }
  // this lane's controlled joint addresses, held across the horizon (read
  // every step; the per-step model launder would otherwise reload them)
  const int ctrl_qa = lane < nc ? m->ctrl_qposadr[lane] : 0, ctrl_da = lane < nc ? m->ctrl_dofadr[lane] : 0;
  PROF_DECL
#if MPCR_PACE
  unsigned* pace = nullptr;
  int pace_own = 0;
  unsigned pace_v = ~0u;
  if ((!WIDE || MPCR_W_PACE) && S::CPW == 1 && WPC == 1 && args.pace) {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // XCC_ID[3:0]
    const unsigned grp = ((((xcc & 7u) * 8u + ((hw >> 13) & 7u)) * 2u + ((hw >> 12) & 1u)) * 16u + ((hw >> 8) & 15u)) *
                             4u + ((hw >> 4) & 3u);
    pace = args.pace + grp * 16u;
    pace_own = (int)(hw & 15u);
  }
#endif
#ifdef MPCR_WAVETIME
  // diagnostic build: per-wave start / end (constant 100 MHz clock), shader
  // cycles and the hardware slot the wave ran on (load-balance study)
  const unsigned long long wt_t0 = __builtin_amdgcn_s_memrealtime(), wt_c0 = __builtin_amdgcn_s_memtime();
  unsigned wt_newton = 0, wt_ls = 0, wt_cvx = 0;  // Newton iterations, line-search passes, convex flush chunks
#endif

  // motion subspaces cdof (lanes over dofs): in the dynamics phase, or --
  // two waves per candidate -- before the first barrier, since the collision
  // wave's constraint rows need them
  auto cdof_phase = [&]() {
    if (lane < nv) {
      const int bd = m->dof_body[lane], kind = m->dof_kind[lane];
      const int tr = m->body_tree[bd];
      float* c = s.cdof[lane];
      float R[9];
#pragma unroll
      for (int k = 0; k < 9; k++) R[k] = s.xmat[bd][k];
      if (kind == 2) {  // free translation
        c[0] = c[1] = c[2] = 0.f;
        const int k = m->dof_sub[lane];
        c[3] = k == 0 ? 1.f : 0.f;
        c[4] = k == 1 ? 1.f : 0.f;
        c[5] = k == 2 ? 1.f : 0.f;
      } else {
        float ax[3], anchor[3];
        if (kind == 3) {
          const int k = m->dof_sub[lane];
          ax[0] = s.xmat[bd][k]; ax[1] = s.xmat[bd][3 + k]; ax[2] = s.xmat[bd][6 + k];  // by index, no selects
          anchor[0] = s.xpos[bd][0]; anchor[1] = s.xpos[bd][1]; anchor[2] = s.xpos[bd][2];
        } else {
          const int j = m->dof_jnt[lane];
          float w[3];
          mv(ax, R, m->jnt_axis[j]);
          mv(w, R, m->jnt_pos[j]);
          anchor[0] = s.xpos[bd][0] + w[0]; anchor[1] = s.xpos[bd][1] + w[1]; anchor[2] = s.xpos[bd][2] + w[2];
        }
        if (kind == 1) {
          c[0] = c[1] = c[2] = 0.f;
          c[3] = ax[0]; c[4] = ax[1]; c[5] = ax[2];
        } else {
          float off[3] = {s.com[tr][0] - anchor[0], s.com[tr][1] - anchor[1], s.com[tr][2] - anchor[2]}, cr[3];
          cross(cr, ax, off);
          c[0] = ax[0]; c[1] = ax[1]; c[2] = ax[2];
          c[3] = cr[0]; c[4] = cr[1]; c[5] = cr[2];
        }
      }
    }
  };
  for (int t = t_begin; t < t_end; t++) {
    // Launder the model pointer every step: otherwise the compiler hoists
    // every loop-invariant model load out of the horizon loop and keeps them
    // all live across the whole step (244 VGPRs + SGPR spills).  The loads
    // stay in their phases and hit L1/L2.
    LAUNDER_MODEL();
    if constexpr ((!WIDE || MPCR_W_LANE_LAUNDER) && MPCR_LANE_LAUNDER) LAUNDER_LANE();
#if MPCR_PACE && MPCR_PACE_AT == 1
    PACE_SETPRIO();  // the previous step's read, against this step
#endif
#if MPCR_PACE
    if (pace) {  // post this step, read the SIMD mates' (consumed mid-step)
      // a plain store keeps the line in this XCD's L2 (agent scope would drop
      // it: every mate's next load then missed L2 -- the launch's largest
      // HBM stream); the readers share the CU, so their L1-bypassing (sc1)
      // loads see it in L2
      if (lane == pace_own) __hip_atomic_store(pace + lane, (unsigned)t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (lane < 16) pace_v = __hip_atomic_load(pace + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#endif
    if (run_main) {  // ---- wave 0 (WPC = 2): joint velocities .. geom poses, eef
    // ---- qvel[:nctrl] = thetadot_t ----------------------------------------------
#if MPCR_TD_TABLE
    if (lane < nc) {
      const float v = vnext;
      if (t + 1 < H) vnext = tdp[lane * H + t + 1];  // next step's, in flight during this one
      s.qvel[ctrl_da] = v;
      if (args.layout != 0 && args.thetadot && live) args.thetadot[(size_t)b * nc * H + lane * H + t] = v;
    }
#else
    if (lane < nc) {
      float v;
      if (args.layout == 0) {
        v = 0.f;
        const float* pd = args.pdot + (size_t)t * args.nbasis;
#pragma unroll
        for (int k = 0; k < 12; k++)
          if (k < args.nbasis) v = fmaf(pd[k], xir[k], v);
      } else {
        v = args.input[(size_t)bi * nc * H + lane * H + t];
      }
      s.qvel[ctrl_da] = v;
      if (args.thetadot && live) args.thetadot[(size_t)b * nc * H + lane * H + t] = v;
    }
#endif
    sync();

    STAMP(0);
    STOP_AT(0)
    LAUNDER_PHASE();  // phase boundary: no cross-phase model-load CSE
    // ---- kinematics: local pose per body, then pointer jumping ----------------
    {
      float q[4] = {1.f, 0.f, 0.f, 0.f}, p[3] = {0.f, 0.f, 0.f};
      int anc = -1;
      if (lane < nb) {
        const int kind = m->body_kind[lane];
        const int j = m->body_jnt[lane];
        q[0] = m->body_bquat[lane][0]; q[1] = m->body_bquat[lane][1];
        q[2] = m->body_bquat[lane][2]; q[3] = m->body_bquat[lane][3];
        p[0] = m->body_bpos[lane][0]; p[1] = m->body_bpos[lane][1]; p[2] = m->body_bpos[lane][2];
        anc = m->body_anc[lane];
        if (kind == BK_FREE) {
          const int a = m->jnt_qposadr[j];
          p[0] = s.qpos[a]; p[1] = s.qpos[a + 1]; p[2] = s.qpos[a + 2];
          q[0] = s.qpos[a + 3]; q[1] = s.qpos[a + 4]; q[2] = s.qpos[a + 5]; q[3] = s.qpos[a + 6];
          float n = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
          if (n < kMinVal) { q[0] = 1.f; q[1] = q[2] = q[3] = 0.f; }
          else { q[0] /= n; q[1] /= n; q[2] /= n; q[3] /= n; }
          anc = -1;
        } else if (kind == BK_HINGE || kind == BK_SLIDE) {
          const float qa = s.qpos[m->jnt_qposadr[j]] - m->jnt_qpos0[j];
          const float* ax = m->jnt_axis[j];
          float R[9];
          q2m(R, q);
          if (kind == BK_SLIDE) {
            float w[3];
            mv(w, R, ax);
            p[0] += w[0] * qa; p[1] += w[1] * qa; p[2] += w[2] * qa;
          } else {
            float sn, cs;
            __sincosf(0.5f * qa, &sn, &cs);
            float qj[4] = {cs, ax[0] * sn, ax[1] * sn, ax[2] * sn}, Rj[9], c[3], rc[3], d[3], w[3];
            c[0] = m->jnt_pos[j][0]; c[1] = m->jnt_pos[j][1]; c[2] = m->jnt_pos[j][2];
            q2m(Rj, qj);
            mv(rc, Rj, c);
            d[0] = c[0] - rc[0]; d[1] = c[1] - rc[1]; d[2] = c[2] - rc[2];
            mv(w, R, d);
            p[0] += w[0]; p[1] += w[1]; p[2] += w[2];
            qmul(q, q, qj);
          }
        }
      }
      for (int r = 0; r < m->jump_rounds; r++) {
        const int src = anc >= 0 ? anc : lane;
        float aq[4], ap[3];
        aq[0] = hshfl<S::CPW>(q[0], src); aq[1] = hshfl<S::CPW>(q[1], src);
        aq[2] = hshfl<S::CPW>(q[2], src); aq[3] = hshfl<S::CPW>(q[3], src);
        ap[0] = hshfl<S::CPW>(p[0], src); ap[1] = hshfl<S::CPW>(p[1], src); ap[2] = hshfl<S::CPW>(p[2], src);
        const int aanc = hshfl<S::CPW>(anc, src);
        if (anc >= 0) {
          float R[9], w[3];
          q2m(R, aq);
          mv(w, R, p);
          p[0] = ap[0] + w[0]; p[1] = ap[1] + w[1]; p[2] = ap[2] + w[2];
          qmul(q, aq, q);
          anc = aanc;
        }
      }
      if (lane < nb) {
        float n = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
        q[0] /= n; q[1] /= n; q[2] /= n; q[3] /= n;
        float R[9], w[3];
        q2m(R, q);
        s.xpos[lane][0] = p[0]; s.xpos[lane][1] = p[1]; s.xpos[lane][2] = p[2];
        s.xquat[lane][0] = q[0]; s.xquat[lane][1] = q[1]; s.xquat[lane][2] = q[2]; s.xquat[lane][3] = q[3];
#pragma unroll
        for (int k = 0; k < 9; k++) s.xmat[lane][k] = R[k];
        mv(w, R, m->body_ipos[lane]);
        s.xipos[lane][0] = p[0] + w[0]; s.xipos[lane][1] = p[1] + w[1]; s.xipos[lane][2] = p[2] + w[2];
      }
    }
    sync();

    STAMP(1);
    STOP_AT(1)
    LAUNDER_PHASE();  // phase boundary: no cross-phase model-load CSE
    // ---- geom poses, tree COMs ------------------------------------------------
    if (lane < m->ngeom) {
      const int gb = m->geom_body[lane];
      float gq[4] = {m->geom_quat[lane][0], m->geom_quat[lane][1], m->geom_quat[lane][2], m->geom_quat[lane][3]};
      float Rg[9];
      q2m(Rg, gq);
      if (gb < 0) {
        s.gxpos[lane][0] = m->geom_pos[lane][0]; s.gxpos[lane][1] = m->geom_pos[lane][1];
        s.gxpos[lane][2] = m->geom_pos[lane][2];
#pragma unroll
        for (int k = 0; k < 9; k++) s.gxmat[lane][k] = Rg[k];
      } else {
        float w[3], R[9], Rr[9];
#pragma unroll
        for (int k = 0; k < 9; k++) R[k] = s.xmat[gb][k];
        mv(w, R, m->geom_pos[lane]);
        s.gxpos[lane][0] = s.xpos[gb][0] + w[0]; s.gxpos[lane][1] = s.xpos[gb][1] + w[1];
        s.gxpos[lane][2] = s.xpos[gb][2] + w[2];
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
          for (int k = 0; k < 3; k++)
            Rr[3 * i + k] = R[3 * i] * Rg[k] + R[3 * i + 1] * Rg[3 + k] + R[3 * i + 2] * Rg[6 + k];
#pragma unroll
        for (int k = 0; k < 9; k++) s.gxmat[lane][k] = Rr[k];
      }
    }
    if constexpr (S::WIDE) {  // connect anchors in world (the body frames die with the dynamics region)
      if (lane < 2 * m->neq && m->eq_type[lane >> 1] == 0) {
        const int e = lane >> 1, side = lane & 1;
        const int bb = side ? m->eq_b2[e] : m->eq_b1[e];
        const float* a = &m->eq_data[e][4 * side];
        float pw[3] = {a[0], a[1], a[2]};
        if (bb >= 0) {
          float R[9], w[3];
#pragma unroll
          for (int k = 0; k < 9; k++) R[k] = s.xmat[bb][k];
          mv(w, R, a);
          pw[0] = s.xpos[bb][0] + w[0]; pw[1] = s.xpos[bb][1] + w[1]; pw[2] = s.xpos[bb][2] + w[2];
        }
        s.eqp[e][side][0] = pw[0]; s.eqp[e][side][1] = pw[1]; s.eqp[e][side][2] = pw[2];
      }
      if (lane < 2 * m->nten) {  // spatial-tendon sites in world
        const int t = lane >> 1, side = lane & 1, bb = m->ten_body[t][side];
        const float* a = m->ten_pos[t][side];
        float pw[3] = {a[0], a[1], a[2]};
        if (bb >= 0) {
          float R[9], w[3];
#pragma unroll
          for (int k = 0; k < 9; k++) R[k] = s.xmat[bb][k];
          mv(w, R, a);
          pw[0] = s.xpos[bb][0] + w[0]; pw[1] = s.xpos[bb][1] + w[1]; pw[2] = s.xpos[bb][2] + w[2];
        }
        s.tenp[t][side][0] = pw[0]; s.tenp[t][side][1] = pw[1]; s.tenp[t][side][2] = pw[2];
      }
    }
    for (int tr = 0; tr < m->ntree; tr++) {
      float mm = (lane < nb && m->body_tree[lane] == tr) ? m->body_mass[lane] : 0.f;
      float cx = hsum<S::CPW>(mm * (lane < nb ? s.xipos[lane][0] : 0.f));
      float cy = hsum<S::CPW>(mm * (lane < nb ? s.xipos[lane][1] : 0.f));
      float cz = hsum<S::CPW>(mm * (lane < nb ? s.xipos[lane][2] : 0.f));
      if (lane == 0) {
        float tm = m->tree_mass[tr];
        s.com[tr][0] = cx / tm; s.com[tr][1] = cy / tm; s.com[tr][2] = cz / tm;
      }
    }
    sync();

    // ---- eef outputs (pre-integration) + pose cost -------------------------
    if (lane == 0) {
      float ep[3] = {0.f, 0.f, 0.f}, eq[4] = {1.f, 0.f, 0.f, 0.f};
      if (m->tcp_body >= 0) {
        float w[3], R[9];
#pragma unroll
        for (int k = 0; k < 9; k++) R[k] = s.xmat[m->tcp_body][k];
        mv(w, R, m->tcp_pos);
        ep[0] = s.xpos[m->tcp_body][0] + w[0]; ep[1] = s.xpos[m->tcp_body][1] + w[1];
        ep[2] = s.xpos[m->tcp_body][2] + w[2];
      }
      if (m->hande_body >= 0) {
        eq[0] = s.xquat[m->hande_body][0]; eq[1] = s.xquat[m->hande_body][1];
        eq[2] = s.xquat[m->hande_body][2]; eq[3] = s.xquat[m->hande_body][3];
      }
      const float* pt = &s.par[PAR_PT];
      const float* qt = &s.par[PAR_QT];
      float dx = ep[0] - pt[0], dy = ep[1] - pt[1], dz = ep[2] - pt[2];
      cost_g += sqrtf(dx * dx + dy * dy + dz * dz);
      float qn = sqrtf(eq[0] * eq[0] + eq[1] * eq[1] + eq[2] * eq[2] + eq[3] * eq[3]);
      float dq = fabsf((eq[0] * qt[0] + eq[1] * qt[1] + eq[2] * qt[2] + eq[3] * qt[3]) / qn);
      cost_r += 2.f * acosf(clampf(dq, -1.f, 1.f));
      if (args.trace_eef && live) {
        float* e = args.trace_eef + ((size_t)b * H + t) * 7;
        e[0] = ep[0]; e[1] = ep[1]; e[2] = ep[2]; e[3] = eq[0]; e[4] = eq[1]; e[5] = eq[2]; e[6] = eq[3];
      }
      if (args.plant && t == H - 1 && live) {
        float* e = args.state + ST_EEF;
        e[0] = ep[0]; e[1] = ep[1]; e[2] = ep[2]; e[3] = eq[0]; e[4] = eq[1]; e[5] = eq[2]; e[6] = eq[3];
      }
    }

    if constexpr (WPC == 2) {
      if (m->coll_rows) cdof_phase();
      sync();
    }
    }  // run_main
    if constexpr (WPC == 2) block_sync();  // geom poses, tree COMs, cdof ready for both waves

    STAMP(2);
    STOP_AT(2)
    LAUNDER_PHASE();  // phase boundary: no cross-phase model-load CSE
    if (run_main) {  // ---- wave 0: the dynamics (cinert .. M^-1 qfrc_smooth)
    // ---- cinert, cdof (+ actuator forces) -------------------------------------
    if constexpr (S::WIDE) {
      if (lane < m->nu) {
        float len = 0.f, vel = 0.f;
        for (int k = 0; k < m->act_ntrn[lane]; k++) {
          len = fmaf(m->act_moment[lane][k], s.qpos[m->act_qadr[lane][k]], len);
          vel = fmaf(m->act_moment[lane][k], s.qvel[m->act_dof[lane][k]], vel);
        }
        const float* g = m->act_gain[lane];
        const float* bp = m->act_bias[lane];
        float gain = g[0];
        if (m->act_gaffine[lane]) gain += g[1] * len + g[2] * vel;
        const float bias = m->act_baffine[lane] ? bp[0] + bp[1] * len + bp[2] * vel : 0.f;
        s.actf[lane] = clampf(gain * g[3] + bias, m->act_frc[lane][0], m->act_frc[lane][1]);
      }
    }
    if (lane < nb) {
      const int tr = m->body_tree[lane];
      float R[9], I[6];
#pragma unroll
      for (int k = 0; k < 9; k++) R[k] = s.xmat[lane][k];
      const float* Il = m->body_Iloc[lane];
      // I_w = R Il R^T
      float A[9] = {Il[0], Il[3], Il[4], Il[3], Il[1], Il[5], Il[4], Il[5], Il[2]}, RA[9];
#pragma unroll
      for (int i = 0; i < 3; i++)
#pragma unroll
        for (int k = 0; k < 3; k++) RA[3 * i + k] = R[3 * i] * A[k] + R[3 * i + 1] * A[3 + k] + R[3 * i + 2] * A[6 + k];
      I[0] = RA[0] * R[0] + RA[1] * R[1] + RA[2] * R[2];
      I[1] = RA[3] * R[3] + RA[4] * R[4] + RA[5] * R[5];
      I[2] = RA[6] * R[6] + RA[7] * R[7] + RA[8] * R[8];
      I[3] = RA[0] * R[3] + RA[1] * R[4] + RA[2] * R[5];
      I[4] = RA[0] * R[6] + RA[1] * R[7] + RA[2] * R[8];
      I[5] = RA[3] * R[6] + RA[4] * R[7] + RA[5] * R[8];
      const float mass = m->body_mass[lane];
      float d[3] = {s.xipos[lane][0] - s.com[tr][0], s.xipos[lane][1] - s.com[tr][1],
                    s.xipos[lane][2] - s.com[tr][2]};
      const float dd = dot3(d, d);
      float* c = s.cinert[lane];
      c[0] = I[0] + mass * (dd - d[0] * d[0]);
      c[1] = I[1] + mass * (dd - d[1] * d[1]);
      c[2] = I[2] + mass * (dd - d[2] * d[2]);
      c[3] = I[3] - mass * d[0] * d[1];
      c[4] = I[4] - mass * d[0] * d[2];
      c[5] = I[5] - mass * d[1] * d[2];
      c[6] = mass * d[0]; c[7] = mass * d[1]; c[8] = mass * d[2];
      c[9] = mass;
    }
    if (WPC == 1 || !m->coll_rows) cdof_phase();
    sync();

    STAMP(3);
    STOP_AT(3)
    LAUNDER_PHASE();  // phase boundary: no cross-phase model-load CSE
    // ---- CRB, velocity, RNE + gravcomp (subtree sums by bitmask) -----------
    constexpr bool MFMA_DYN = NVW == 16 && NBW == 16 && S::CPW == 1 && MPCR_MFMA_DYN;
    float* dscr = &s.xquat[0][0];  // xquat + xmat (256 floats) are dead after the cdof phase
    if constexpr (MFMA_DYN) {
      const int mr = lane & 15, kq = lane >> 4;
      const float* qv = s.qvel;
      const mfx4 z4 = {0.f, 0.f, 0.f, 0.f};
      // crb[b] = sum of cinert over b's subtree
      {
        const uint32_t sub = mr < nb ? m->body_submask[mr] : 0u;
        const mfx4 acc = mm16<4>([&](int, int k) { return ((sub >> k) & 1u) ? 1.f : 0.f; },
                                 [&](int k, int j) { return (k < nb && j < 10) ? s.cinert[k][j] : 0.f; }, z4, lane);
#pragma unroll
        for (int v = 0; v < 4; v++)
          if (4 * kq + v < nb && mr < 10) s.crb[4 * kq + v][mr] = acc[v];
      }
      // cvel[b] = sum over b's chain of qvel x cdof; the velocity before each
      // dof (its velmask) likewise, into the scratch for cdof_dot
      {
        const uint32_t bm = mr < nb ? m->body_dofmask[mr] : 0u, vm = mr < nv ? m->dof_velmask[mr] : 0u;
        mfx4 cv = z4, vv = z4;
#pragma unroll
        for (int s4 = 0; s4 < 4; s4++) {
          const int k = 4 * s4 + kq;
          const float q = k < nv ? qv[k] : 0.f;
          const float bcd = (k < nv && mr < 6) ? s.cdof[k][mr] : 0.f;
          cv = __builtin_amdgcn_mfma_f32_16x16x4f32(((bm >> k) & 1u) ? q : 0.f, bcd, cv, 0, 0, 0);
          vv = __builtin_amdgcn_mfma_f32_16x16x4f32(((vm >> k) & 1u) ? q : 0.f, bcd, vv, 0, 0, 0);
        }
#pragma unroll
        for (int v = 0; v < 4; v++) {
          if (4 * kq + v < nb && mr < 6) s.cvel[4 * kq + v][mr] = cv[v];
          if (mr < 6) dscr[(4 * kq + v) * 8 + mr] = vv[v];
        }
      }
      sync();
      if (lane < nv) {  // cdof_dot = cvel_before x cdof (0 for free translation)
        float v[6], r[6];
#pragma unroll
        for (int k = 0; k < 6; k++) v[k] = dscr[lane * 8 + k];
        cross_motion(r, v, s.cdof[lane]);
        const bool zero = m->dof_kind[lane] == 2;
#pragma unroll
        for (int k = 0; k < 6; k++) s.cdofdot[lane][k] = zero ? 0.f : r[k];
      }
      sync();
      // RNE accelerations: (0, -g) + sum over the chain of qvel x cdof_dot
      {
        const uint32_t bm = mr < nb ? m->body_dofmask[mr] : 0u;
        mfx4 a4;
#pragma unroll
        for (int v = 0; v < 4; v++) a4[v] = (mr >= 3 && mr < 6) ? -m->gravity[mr - 3] : 0.f;
        a4 = mm16<4>([&](int, int k) { return ((bm >> k) & 1u) ? (k < nv ? qv[k] : 0.f) : 0.f; },
                     [&](int k, int j) { return (k < nv && j < 6) ? s.cdofdot[k][j] : 0.f; }, a4, lane);
#pragma unroll
        for (int v = 0; v < 4; v++)
          if (mr < 6) dscr[128 + (4 * kq + v) * 8 + mr] = a4[v];
      }
    } else {
    for (int idx = lane; idx < nb * 10; idx += S::HL) {
      const int bb = idx / 10, k = idx - bb * 10;
      uint32_t sm = m->body_submask[bb];
      float acc = 0.f;
      while (sm) {
        const int c = __builtin_ctz(sm);
        sm &= sm - 1;
        acc += s.cinert[c][k];
      }
      s.crb[bb][k] = acc;
    }
    if (lane < nb) {  // cvel = sum over the chain of cdof * qvel
      uint32_t dm = m->body_dofmask[lane];
      float v[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      while (dm) {
        const int d = __builtin_ctz(dm);
        dm &= dm - 1;
        const float qd = s.qvel[d];
#pragma unroll
        for (int k = 0; k < 6; k++) v[k] = fmaf(s.cdof[d][k], qd, v[k]);
      }
#pragma unroll
      for (int k = 0; k < 6; k++) s.cvel[lane][k] = v[k];
    }
    if (lane < nv) {  // cdof_dot = cvel_before x cdof (0 for free translation)
      uint32_t dm = m->dof_velmask[lane];
      float v[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, r[6];
      while (dm) {
        const int d = __builtin_ctz(dm);
        dm &= dm - 1;
        const float qd = s.qvel[d];
#pragma unroll
        for (int k = 0; k < 6; k++) v[k] = fmaf(s.cdof[d][k], qd, v[k]);
      }
      cross_motion(r, v, s.cdof[lane]);
      const bool zero = m->dof_kind[lane] == 2;
#pragma unroll
      for (int k = 0; k < 6; k++) s.cdofdot[lane][k] = zero ? 0.f : r[k];
    }
    }
    sync();
    if (lane < nv) {  // f_i = crb[body(i)] * cdof_i
      float f[6];
      mul_inert_vec(f, s.crb[m->dof_body[lane]], s.cdof[lane]);
#pragma unroll
      for (int k = 0; k < 6; k++) s.fvec[lane][k] = f[k];
    }
    if (lane < nb) {  // cfrc_body = I*cacc + v x* (I v) - gravcomp wrench
      float a[6];
      if constexpr (MFMA_DYN) {
#pragma unroll
        for (int k = 0; k < 6; k++) a[k] = dscr[128 + lane * 8 + k];
      } else {
        uint32_t dm = m->body_dofmask[lane];
        a[0] = a[1] = a[2] = 0.f;
        a[3] = -m->gravity[0]; a[4] = -m->gravity[1]; a[5] = -m->gravity[2];
        while (dm) {
          const int d = __builtin_ctz(dm);
          dm &= dm - 1;
          const float qd = s.qvel[d];
#pragma unroll
          for (int k = 0; k < 6; k++) a[k] = fmaf(s.cdofdot[d][k], qd, a[k]);
        }
      }
      float f[6], iv[6], vf[6], cv[6];
#pragma unroll
      for (int k = 0; k < 6; k++) cv[k] = s.cvel[lane][k];
      mul_inert_vec(f, s.cinert[lane], a);
      mul_inert_vec(iv, s.cinert[lane], cv);
      cross_force(vf, cv, iv);
      const float gc = m->body_gravcomp[lane] * m->body_mass[lane];
      const int tr = m->body_tree[lane];
      float F[3] = {-m->gravity[0] * gc, -m->gravity[1] * gc, -m->gravity[2] * gc};
      float rr[3] = {s.xipos[lane][0] - s.com[tr][0], s.xipos[lane][1] - s.com[tr][1],
                     s.xipos[lane][2] - s.com[tr][2]}, tq[3];
      float Tv[3] = {0.f, 0.f, 0.f};
      if constexpr (S::WIDE) {  // inertia-box viscosity at xipos: v = v_com + w x rr
        const float vl = m->body_visc[lane][0], va = m->body_visc[lane][1];
        float wr[3];
        cross(wr, cv, rr);
#pragma unroll
        for (int k = 0; k < 3; k++) { F[k] += vl * (cv[3 + k] + wr[k]); Tv[k] = va * cv[k]; }
      }
      cross(tq, rr, F);
      tq[0] += Tv[0]; tq[1] += Tv[1]; tq[2] += Tv[2];
      s.cfrc[lane][0] = f[0] + vf[0] - tq[0];
      s.cfrc[lane][1] = f[1] + vf[1] - tq[1];
      s.cfrc[lane][2] = f[2] + vf[2] - tq[2];
      s.cfrc[lane][3] = f[3] + vf[3] - F[0];
      s.cfrc[lane][4] = f[4] + vf[4] - F[1];
      s.cfrc[lane][5] = f[5] + vf[5] - F[2];
    }
    sync();
    STAMP(4);
    STOP_AT(4)
    LAUNDER_PHASE();  // phase boundary: no cross-phase model-load CSE
    // mass matrix entries (chain-masked) + bias forces
    if constexpr (MFMA_DYN) {
      // P = fvec cdof^T (K = 6 in two instructions); M[i][j] = P[i][j] for j on
      // i's chain, mirrored to M[j][i]; the bias forces' subtree sums of cfrc
      const int mr = lane & 15, kq = lane >> 4;
      const mfx4 z4 = {0.f, 0.f, 0.f, 0.f};
      const mfx4 P = mm16<2>([&](int i, int c) { return (i < nv && c < 6) ? s.fvec[i][c] : 0.f; },
                             [&](int c, int j) { return (j < nv && c < 6) ? s.cdof[j][c] : 0.f; }, z4, lane);
      const int j = mr;
#pragma unroll
      for (int v = 0; v < 4; v++) {
        const int i = 4 * kq + v;
        if (i < nv && j < nv) {
          if ((m->dof_chainmask[i] >> j) & 1u) {
            const float x = i == j ? P[v] + m->dof_armature[i] : P[v];
            m_set(i, j, x);
            m_set(j, i, x);
          } else if (!((m->dof_chainmask[j] >> i) & 1u)) {
            m_set(i, j, 0.f);
          }
        } else {
          m_set(i, j, i == j ? 1.f : 0.f);
        }
      }
      const uint32_t sub = mr < nv ? m->dof_submask[mr] : 0u;
      const mfx4 fb = mm16<4>([&](int, int b) { return ((sub >> b) & 1u) ? 1.f : 0.f; },
                              [&](int b, int c) { return (b < nb && c < 6) ? s.cfrc[b][c] : 0.f; }, z4, lane);
#pragma unroll
      for (int v = 0; v < 4; v++)
        if (mr < 6) dscr[(4 * kq + v) * 8 + mr] = fb[v];
      sync();
    } else {
    for (int idx = lane; idx < NVW * NVW; idx += S::HL) {
      const int i = idx >> S::LOG_NVW, j = idx & (NVW - 1);
      float v = 0.f;
      if (i < nv && j < nv) {
        if ((m->dof_chainmask[i] >> j) & 1u) {
#pragma unroll
          for (int k = 0; k < 6; k++) v = fmaf(s.cdof[j][k], s.fvec[i][k], v);
        } else if ((m->dof_chainmask[j] >> i) & 1u) {
#pragma unroll
          for (int k = 0; k < 6; k++) v = fmaf(s.cdof[i][k], s.fvec[j][k], v);
        }
        if (i == j) v += m->dof_armature[i];
      } else if (i == j) {
        v = 1.f;
      }
      m_set(i, j, v);
    }
    }
    if (lane < nv) {
      float f[6];
      if constexpr (MFMA_DYN) {
#pragma unroll
        for (int k = 0; k < 6; k++) f[k] = dscr[lane * 8 + k];
      } else {
      uint32_t sm = m->dof_submask[lane];
      f[0] = f[1] = f[2] = f[3] = f[4] = f[5] = 0.f;
      while (sm) {
        const int c = __builtin_ctz(sm);
        sm &= sm - 1;
#pragma unroll
        for (int k = 0; k < 6; k++) f[k] += s.cfrc[c][k];
      }
      }
      float bias = 0.f;
#pragma unroll
      for (int k = 0; k < 6; k++) bias = fmaf(s.cdof[lane][k], f[k], bias);
      float qf = -bias - m->dof_damping[lane] * s.qvel[lane];
      if constexpr (S::WIDE) {
        if (m->has_spring) qf -= m->dof_stiffness[lane] * (s.qpos[m->dof_qposadr[lane]] - m->dof_springref[lane]);
        float fa = 0.f;
        for (int k = 0; k < m->dof_actn[lane]; k++) fa = fmaf(m->dof_actm[lane][k], s.actf[m->dof_acta[lane][k]], fa);
        qf += clampf(fa, m->dof_actfrc[lane][0], m->dof_actfrc[lane][1]);
      }
      s.qfs[lane] = qf;
    } else if (lane < NVW) {
      s.qfs[lane] = 0.f;
    }
    sync();

    STAMP(5);
    STOP_AT(5)
    LAUNDER_PHASE();  // phase boundary: no cross-phase model-load CSE
    // ---- qacc_smooth = M^-1 qfrc_smooth (row-per-lane Cholesky) -------------
    if (S::CPW == 1 && blk_usable<NVW>(m)) {
      // M is block diagonal by kinematic tree: one chain for all trees
      if (lane >= nv && lane < NVW) s.qas[lane] = 0.f;
      blk_solve<NVW>(m, [&](int i, int j) { return m_get(i, j); }, s.qfs, s.qas, lane, &s.xpos[0][0]);
    } else {
      float Lm[NVW];
#pragma unroll
      for (int j = 0; j < NVW; j++) Lm[j] = lane < NVW ? m_get(lane, j) : 0.f;
      // the dynamics region (xpos..fvec) is dead once M is assembled
      float x;
      if constexpr (NVW == 16 && MPCR_DPP_CHOL) {
        float dinv;
        chol16(Lm, dinv, lane);
        x = chol16_solve<S::LD>(Lm, dinv, lane < NVW ? s.qfs[lane] : 0.f, lane, &s.xpos[0][0]);
      } else {
        chol_rows(Lm, lane);
        x = chol_solve<NVW, S::LD>(Lm, lane < NVW ? s.qfs[lane] : 0.f, lane, &s.xpos[0][0]);
      }
      if (lane < NVW) s.qas[lane] = lane < nv ? x : 0.f;
    }

    }  // run_main (dynamics)

    STAMP(6);
    STOP_AT(6)
#if MPCR_PACE && MPCR_PACE_AT == 0
    PACE_SETPRIO();
#endif
    LAUNDER_PHASE();  // phase boundary: no cross-phase model-load CSE
    // Swap mode (two waves, dual-arm class without cost slots, round 5): the
    // collision wave only culls the pairs and lists the convex ones, posts
    // the list (an LDS step token, no barrier) and goes on to their MPRs (the
    // lead flush below); wave 0, after the dynamics, runs the other pairs'
    // narrow phase, so both waves reach the manifold queue together.  The
    // contacts keep the one-wave order (these pairs' first, chunk by chunk,
    // then the convex ones).  With more convex pairs than the lead flush
    // takes, the collision wave runs that narrow phase itself, as before.
    const bool swapm = WPC == 2 && S::WIDE && MPCR_W2_SWAP && MPCR_W2_LEAD && m->cvx_joint && m->nslot == 0;
    for (int pass = 0; pass < 2 && (run_coll || swapm); pass++) {
    bool do_list = false, do_narrow = false;
    if (run_coll) {
      if (pass == 0) { do_list = true; do_narrow = !swapm; }
      else do_narrow = swapm && s.ncvx > m->w2_lead_max;
    } else if (pass == 1) {  // wave 0 (swap mode): the list is posted for this step
      bool posted = true;
      if constexpr (S::SPLIT) {  // (bounded: a lost post flags the candidate instead of hanging the launch)
        int guard = 0;
        while (__hip_atomic_load(&s.ctok_[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != t + 1 &&
               ++guard < (1 << 22))
          __builtin_amdgcn_s_sleep(1);
        // a lost post: its own status bit (MPCR_STATUS_SYNC, the outputs are
        // void), and the list is not read -- wave 1 may still be writing it
        if (guard >= (1 << 22)) { status |= 1 << 10; posted = false; }
      }
      do_narrow = posted && s.ncvx <= m->w2_lead_max;
    }
    if (do_list || do_narrow) {
    // ---- collision: lanes over pairs (typed segments); cost_c on the masked
    //      slots; active contacts compacted into the list; box-box pairs
    //      that pass the bounding-sphere cull are solved wave-cooperatively
    if (do_list) {
      if (lane == 0) { s.ncon = 0; s.ncvx = 0; }
      sync();
    }
    // (the general-convex pairs are sorted last, from DevModel::cvx_base: a
    // list-only pass starts at their chunk, a narrow-only pass ends there)
    const int k_lo = do_narrow ? 0 : m->cvx_base / S::HL, p_hi = do_list ? m->npair : min(m->npair, m->cvx_base);
    for (int k = k_lo; k * S::HL < p_hi; k++) {
      const int p = lane + k * S::HL;
      const bool valid = p < m->npair;
      const int func = valid ? m->pair_func[p] : -1;
      const bool defer = S::WIDE && func >= 9;  // general convex: the list
      bool run = valid && (defer ? do_list : do_narrow);
      if (run && m->pair_slotadr[p] < 0) {
        const int g1 = m->pair_g1[p], g2 = m->pair_g2[p];
        const float dx = s.gxpos[g2][0] - s.gxpos[g1][0], dy = s.gxpos[g2][1] - s.gxpos[g1][1],
                    dz = s.gxpos[g2][2] - s.gxpos[g1][2];
        if (m->geom_type[g1] != 0) {
          run = sqrtf(dx * dx + dy * dy + dz * dz) <= m->geom_rbound[g1] + m->geom_rbound[g2] + m->pair_margin[p];
          if constexpr (S::WIDE) {  // box vs the other geom's bounding sphere (exact cull, as the oracle)
            if (run && func == 9 && (m->geom_type[g1] == 6 || m->geom_type[g2] == 6)) {
              const bool b1 = m->geom_type[g1] == 6;
              const int gb = b1 ? g1 : g2;
              const float sg = b1 ? 1.f : -1.f;
              float d[3] = {sg * dx, sg * dy, sg * dz}, l[3];
              mtv(l, s.gxmat[gb], d);
              float o2 = 0.f;
#pragma unroll
              for (int k2 = 0; k2 < 3; k2++) {
                const float e = fmaxf(fabsf(l[k2]) - m->geom_size[gb][k2], 0.f);
                o2 += e * e;
              }
              run = sqrtf(o2) <= m->geom_rbound[b1 ? g2 : g1] + m->pair_margin[p];
            }
          }
        } else {  // plane vs the other geom's bounding sphere (C3: the box far above the floor)
          const float* R1 = s.gxmat[g1];
          run = R1[2] * dx + R1[5] * dy + R1[8] * dz <= m->geom_rbound[g2] + m->pair_margin[p];
        }
      }
      // general convex pairs (sorted last) that survive the cull are compacted
      // into a list and solved 64 at a time below, instead of leaving most
      // lanes of every 64-pair chunk idle behind a few MPR lanes
      if (S::WIDE && do_list) {
        const unsigned long long dm = __ballot(defer && run);
        if (defer && run) s.cvx[s.ncvx + lanes_below(dm)] = p;
        sync();
        if (lane == 0) s.ncvx += __popcll(dm);
      }
      if (!do_narrow) continue;
      float dist[4] = {1e30f, 1e30f, 1e30f, 1e30f}, pos[4][3] = {}, nrm[4][3] = {};
      int nsl = 0;
      if (run && func != 4 && !defer && !(MPCR_ABL_FUNC & (1 << func))) nsl = narrow_lane(m, s, hx, p, dist, pos, nrm);
      STAMP(11);
      const unsigned long long bbm = hballot<S::CPW>(run && func == 4 && !(MPCR_ABL_FUNC & 16));
      emit_contacts(m, s, args, b, t, H, valid && func != 4 && !defer, p, nsl, dist, pos, nrm, cost_c, shist, k);
      STAMP(12);
      if (bbm && !(m->disableflags & 16)) {
        unsigned long long mm = bbm;
        while (mm) {
          const int q = __builtin_ctzll(mm);
          mm &= mm - 1;
          box_box_wave(m, s, k * S::HL + q - hbase<S::CPW>(), lane);
        }
      }
      STAMP(16);
    }
    if constexpr (!S::WIDE) {
      if (s.ncon > S::MAXACT) {
        status |= 1;
        sync();
        if (lane == 0) s.ncon = S::MAXACT;
        sync();
      }
    }
    }  // do_list || do_narrow
    if constexpr (S::SPLIT) {
      if (swapm && run_coll && pass == 0) {  // post the list (every lane's entries first)
        sync();
        if (lane == 0) __hip_atomic_store(&s.ctok_[0], t + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    }  // pass
    if constexpr (S::WIDE) {
      // ---- the convex flush: every general-convex pair that survived the
      //      cull (the list holds all of a model's, so this is the step's only
      //      flush), MPR per lane, then the pending manifolds wave-cooperatively
      //      one pair at a time.  Two waves per candidate (round 5): the
      //      dynamics wave joins after the mass-matrix solve and the pairs are
      //      dealt over both (item i on wave i & 1, rounds of 128), each wave
      //      running the manifolds of its own pairs with its own clip scratch;
      //      the contacts go to the list in pair order (a prefix over both
      //      waves' counts), so the list -- and every result -- is bitwise the
      //      one-wave kernel's.  Models with cost slots on convex pairs keep
      //      the flush on the collision wave (cost_c accumulates per lane).
      const bool split = WPC == 2 && m->cvx_joint;
      const bool mine = WPC == 1 || split || wv == 1;
      PolyScratchT<S::PMAXW>* const psc = reinterpret_cast<PolyScratchT<S::PMAXW>*>(
          (WPC == 2 && wv == 0) ? &s.xpos[0][0] : &s.polyw[0][0][0]);
      int* const jcnt = reinterpret_cast<int*>(&s.xpos[0][0]) + sizeof(PolyScratchT<S::PMAXW>) / 4;
      // Lead flush (two waves, round 5): with at most W2_LEAD_MAX pairs in the
      // list, the collision wave runs every pair's MPR (one lane each) as soon
      // as its list is complete -- while wave 0 still runs the dynamics --
      // and queues the polyhedron manifolds; after the hand-over both waves
      // take manifolds from the queue (an LDS counter), wave 0 returning its
      // results through a mailbox in the dead dynamics region, and the
      // collision wave emits the contacts in pair order.  Each pair's MPR and
      // manifold are the same instructions on the same data wherever they
      // run: bitwise the one-wave kernel.
      int* const jq = reinterpret_cast<int*>(&s.cvx[0]);  // [0] next job, [1] jobs, records from [2]
      float* const mbox = reinterpret_cast<float*>(jcnt);  // wave 0's manifold results, W2_JOB_OUT floats per job
      int lpc = 0, ljob = 0, lsl = 0;
      float ld[4] = {1e30f, 1e30f, 1e30f, 1e30f}, lp[4][3] = {}, ln[4][3] = {};
      if (MPCR_W2_LEAD && split && wv == 1 && s.ncvx <= m->w2_lead_max) {
        const bool v = lane < s.ncvx;
        lpc = v ? s.cvx[lane] : 0;
        lsl = v ? narrow_lane(m, s, hx, lpc, ld, lp, ln, (args.dbg && b == 0 && t == H - 1) ? args.dbg : nullptr)
                : 0;
        STAMP(21);
        for (unsigned long long pm = __ballot(lsl == kPendingManifold); pm; pm &= pm - 1) {
          const int q = __builtin_ctzll(pm);
          const int pq = __shfl(lpc, q);
          const float dq = __shfl(ld[0], q);
          const int gp = m->pair_g1[pq];
          const float* Rp = s.gxmat[gp];
          const float nq[3] = {Rp[2], Rp[5], Rp[8]};
          plane_mesh_manifold_wave(m, s, m->pair_g2[pq], nq, s.gxpos[gp], -dq, q, lane, ld, lp, ln, lsl);
        }
        STAMP(22);
        // the manifold queue: (pair | lane << 16, MPR depth, normal, point) per job
        const unsigned long long pm = __ballot(lsl == kPendingPoly);
        ljob = lanes_below(pm);
        if (lsl == kPendingPoly) {
          int* r = jq + 2 + W2_JOB_REC * ljob;
          r[0] = lpc | (lane << 16);
          r[1] = __float_as_int(ld[0]);
#pragma unroll
          for (int e = 0; e < 3; e++) { r[2 + e] = __float_as_int(ln[0][e]); r[5 + e] = __float_as_int(lp[0][e]); }
        }
        if (lane == 0) { jq[0] = 0; jq[1] = __popcll(pm); }
      }
      if constexpr (WPC == 2) block_sync();  // the list is complete; the dynamics are done
      const int ncv = s.ncvx, rstep = split ? 2 * WAVE : WAVE;
      const bool lead = MPCR_W2_LEAD && split && ncv <= m->w2_lead_max;
      int ncon_w = s.ncon;
      if (lead) {
        STAMP(16);  // (profile build: wave 0's wait for the queue)
        const int njob = jq[1];
        for (;;) {
          int j = 0;
          if (lane == 0) j = __hip_atomic_fetch_add(jq, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          j = __builtin_amdgcn_readfirstlane(j);
          if (j >= njob) break;
          const int* r = jq + 2 + W2_JOB_REC * j;
          const int pq = r[0] & 0xffff, q = r[0] >> 16;
          const float dq = __int_as_float(r[1]);
          const float nq[3] = {__int_as_float(r[2]), __int_as_float(r[3]), __int_as_float(r[4])};
          if (wv == 0) {  // lane q stands in for the collision wave's lane q
            lsl = lane == q ? kPendingPoly : 0;
            ld[0] = dq; ld[1] = ld[2] = ld[3] = 1e30f;
#pragma unroll
            for (int e = 0; e < 3; e++) { ln[0][e] = nq[e]; lp[0][e] = __int_as_float(r[5 + e]); }
          }
          poly_manifold_wave(m, s, *psc, hx, pq, nq, -dq, q, lane, ld, lp, ln, lsl);
          if (wv == 0 && lane == q) {
            float* o = mbox + W2_JOB_OUT * j;
#pragma unroll
            for (int c = 0; c < 4; c++) {
              o[c] = ld[c];
#pragma unroll
              for (int e = 0; e < 3; e++) { o[4 + 3 * c + e] = lp[c][e]; o[16 + 3 * c + e] = ln[c][e]; }
            }
            o[28] = __int_as_float(lsl);
          }
        }
        STAMP(17);
        block_sync();  // every manifold done
        if (wv == 1) {
          if (lsl == kPendingPoly) {  // run by wave 0
            const float* o = mbox + W2_JOB_OUT * ljob;
#pragma unroll
            for (int c = 0; c < 4; c++) {
              ld[c] = o[c];
#pragma unroll
              for (int e = 0; e < 3; e++) { lp[c][e] = o[4 + 3 * c + e]; ln[c][e] = o[16 + 3 * c + e]; }
            }
            lsl = __float_as_int(o[28]);
          }
          emit_contacts(m, s, args, b, t, H, lane < ncv, lpc, lsl, ld, lp, ln, cost_c, shist, -1);
        }
        STAMP(18);
      }
      for (int i0 = 0; !lead && i0 < ncv; i0 += rstep) {
#ifdef MPCR_WAVETIME
        wt_cvx++;
#endif
        const int i = split ? i0 + 2 * lane + wv : i0 + lane;
        const bool v = mine && i < ncv;
        const int pc = v ? s.cvx[i] : 0;
        float cd[4] = {1e30f, 1e30f, 1e30f, 1e30f}, cp[4][3] = {}, cn[4][3] = {};
        int cn_sl = v ? narrow_lane(m, s, hx, pc, cd, cp, cn, (args.dbg && b == 0 && t == H - 1) ? args.dbg
                                                                                           : nullptr)
                      : 0;
        STAMP(21);
        for (unsigned long long pm = __ballot(cn_sl == kPendingManifold); pm; pm &= pm - 1) {
          const int q = __builtin_ctzll(pm);  // penetrating plane-mesh pairs, one at a time, all lanes
          const int pq = __shfl(pc, q);
          const float dq = __shfl(cd[0], q);
          const int gp = m->pair_g1[pq];
          const float* Rp = s.gxmat[gp];
          const float nq[3] = {Rp[2], Rp[5], Rp[8]};
          plane_mesh_manifold_wave(m, s, m->pair_g2[pq], nq, s.gxpos[gp], -dq, q, lane, cd, cp, cn, cn_sl);
        }
        STAMP(22);
        for (unsigned long long pm = __ballot(cn_sl == kPendingPoly); pm; pm &= pm - 1) {
          const int q = __builtin_ctzll(pm);  // penetrating polyhedron pairs, one at a time, all lanes
          const int pq = __shfl(pc, q);
          const float dq = __shfl(cd[0], q);
          const float nq[3] = {__shfl(cn[0][0], q), __shfl(cn[0][1], q), __shfl(cn[0][2], q)};
          poly_manifold_wave(m, s, *psc, hx, pq, nq, -dq, q, lane, cd, cp, cn, cn_sl);
        }
        STAMP(17);
        if (split) {
          // this item's active contacts; their list offsets from both waves'
          // counts in item order (lane l holds items 2l and 2l + 1)
          int act = 0;
          if (v && !(m->disableflags & 16)) {
            const float mg = m->pair_margin[pc];
#pragma unroll
            for (int c = 0; c < 4; c++) act += (c < cn_sl && cd[c] < mg) ? 1 : 0;
          }
          jcnt[2 * lane + wv] = act;
          block_sync();
          const int a0 = jcnt[2 * lane], a1 = jcnt[2 * lane + 1];
          int tot;
          const int pre = wscan_excl<4>(a0 + a1, tot) + (wv ? a0 : 0);  // two items: up to 8
          if (act) put_contacts(m, s, ncon_w + pre, pc, cn_sl, cd, cp, cn);
          ncon_w += tot;
          block_sync();  // jcnt is the next round's
        } else if (mine) {
          emit_contacts(m, s, args, b, t, H, v, pc, cn_sl, cd, cp, cn, cost_c, shist, -1);
        }
        STAMP(18);
      }
      if (split && !lead && run_coll && lane == 0) s.ncon = ncon_w;
      sync();
      if (run_coll && s.ncon > S::MAXACT) {
        status |= 1;
        sync();
        if (lane == 0) s.ncon = S::MAXACT;
        sync();
      }
    }
    // WPC = 2 and DevModel::coll_rows: the collision wave builds the
    // constraint rows too, still beside wave 0's dynamics (they need the
    // contacts, qpos, qvel, cdof and the tree COMs, all ready before the first
    // barrier) and hands them over at the second; otherwise wave 0 builds them
    // after the contact list is handed over
    const bool rows_c = WPC == 2 && m->coll_rows;
    // two waves per candidate, dual-arm class, rows after the hand-over (round
    // 5): both waves build the constraint rows, the Jacobian entries and the
    // row parameters dealt over 128 lanes (the bookkeeping -- row counts,
    // sources, offsets -- computed identically on both), and wave 1 leaves at
    // the barrier that follows; same values in the same places as one wave
    const bool rows_j = WPC == 2 && S::WIDE && !rows_c;
    // ... and wave 1 then builds the Newton Hessians (round 5)
    const bool hess2 = MPCR_W2_HESS && rows_j && NVW == 32 && S::CPW == 1;
    // ... and factors the implicit solve's M + dt D (blocked path) for wave 0
    // to sweep after Newton: the factor needs only M, wave 1 is otherwise
    // idle then, and its element gather was most of the solve's time
    const bool impl2 = MPCR_W2_IMPL && hess2 && S::WIDE && m->integrator == 3 && !m->impl_cross && blk_usable<NVW>(m);
    constexpr int BLK_N = NVW == 16 ? 8 : 16;
    static_assert(!S::SPLIT || (BLK_N + 1) * WAVE <= S::DYN_FLOATS, "the implicit factor inside the dynamics region");
    float* const implf = &s.xpos[0][0];  // the factor: BLK_N + 1 floats per lane (dynamics region, dead until Euler)
    const int rl0 = rows_j ? wv * S::HL : 0, rls = rows_j ? 2 * S::HL : S::HL;
    if constexpr (WPC == 2) {
      if (!rows_c) {
        block_sync();  // the contact list is ready; wave 1 waits for the next step's geom poses
        if (!run_main && !rows_j) continue;
      }
    }

    STAMP(7);
    STOP_AT(7)
    LAUNDER_PHASE();  // phase boundary: no cross-phase model-load CSE
    // ---- constraint rows: equality, limits, contacts ------------------------
    bool coupled = true;  // a constraint row spans two kinematic trees (Newton's H not block diagonal)
    if (WPC == 1 || rows_j || (rows_c ? run_coll : run_main)) {
      const int ncon = s.ncon;
      const int neq = (m->disableflags & 64) ? 0 : (S::WIDE ? m->neqrow : m->neq);
      int nlim_l = 0, lsides = 0;
      if (lane < m->njnt && !(m->disableflags & 32) && m->jnt_limited[lane] &&
          (m->jnt_type[lane] == 2 || m->jnt_type[lane] == 3)) {
        const float q = s.qpos[m->jnt_qposadr[lane]];
        if (q - m->jnt_range[lane][0] < m->jnt_margin[lane]) { nlim_l++; lsides |= 1; }
        if (m->jnt_range[lane][1] - q < m->jnt_margin[lane]) { nlim_l++; lsides |= 2; }
      }
      int nlim;
      const int lim_pre = hscan_excl<S::CPW>(nlim_l, nlim);
      // spatial-tendon limit rows after the joint limits (wave-uniform)
      int ntr = 0, tsides = 0;
      if constexpr (S::WIDE) {
        if (!(m->disableflags & 32))
          for (int t = 0; t < m->nten; t++) {
            if (!m->ten_limited[t]) continue;
            const float dx = s.tenp[t][1][0] - s.tenp[t][0][0], dy = s.tenp[t][1][1] - s.tenp[t][0][1],
                        dz = s.tenp[t][1][2] - s.tenp[t][0][2];
            const float len = sqrtf(dx * dx + dy * dy + dz * dz);
            if (len - m->ten_range[t][0] < m->ten_margin[t]) { tsides |= 1 << (2 * t); ntr++; }
            if (m->ten_range[t][1] - len < m->ten_margin[t]) { tsides |= 2 << (2 * t); ntr++; }
          }
      }
      const bool ell = S::WIDE && m->cone == 1;
      int ncr = 0;
      if (lane < ncon) ncr = m->pair_condim[s.con_pair[lane]] == 1 ? 1 : (ell ? 3 : 4);
      int ncrow;
      const int con_pre = hscan_excl<S::CPW>(ncr, ncrow);
      int nefc = neq + nlim + ntr + ncrow;
      int keep_con = ncon;
      if (nefc > S::MAXEFC) {  // keep the longest prefix of contacts that fits
        const int room = S::MAXEFC - neq - nlim - ntr;
        const unsigned long long fit = hballot<S::CPW>(lane < ncon && con_pre + ncr <= room);
        keep_con = __popcll(fit);
        nefc = neq + nlim + ntr + (keep_con > 0 ? hshfl<S::CPW>(con_pre + ncr, keep_con - 1) : 0);
        status |= 1;
      }
      // equality rows: joint (side 0) or connect component side - 1
      if (lane < neq)
        s.efc_src[lane] = S::WIDE ? ((1 << 24) | (m->eqrow_eq[lane] << 4) | m->eqrow_k[lane]) : ((1 << 24) | (lane << 4));
      if (nlim_l) {
        int o = neq + lim_pre;
        if (lsides & 1) s.efc_src[o++] = (2 << 24) | (lane << 4) | 0;
        if (lsides & 2) s.efc_src[o++] = (2 << 24) | (lane << 4) | 1;
      }
      if constexpr (S::WIDE) {
        if (lane == 0 && ntr) {
          int o = neq + nlim;
          for (int t = 0; t < m->nten; t++)
            for (int side = 0; side < 2; side++)
              if ((tsides >> (2 * t + side)) & 1) s.efc_src[o++] = (4 << 24) | (t << 4) | side;
        }
      }
      if (lane < keep_con) {
        const int o = neq + nlim + ntr + con_pre;
        s.con_row[lane] = o;
        if (ncr == 3) {  // elliptic (wide variant only)
          const int p = s.con_pair[lane];
          for (int r = 0; r < 3; r++) s.efc_src[o + r] = (5 << 24) | (lane << 14) | (p << 4) | r;
        } else {
          for (int r = 0; r < ncr; r++) s.efc_src[o + r] = (3 << 24) | (lane << 4) | r;
        }
      }
      {
        bool cross = false;
        if (lane < keep_con) {
          const int4 ji = m->pair_jinfo[s.con_pair[lane]];
          cross = ji.x != 0 && ji.y != 0 && ji.z != ji.w;
        }
        coupled = m->eq_cross || hballot<S::CPW>(cross) != 0ull;
      }
      if (lane == 0) s.nefc = nefc;
      sync();
      // Jacobian entries of equality/limit rows: (row, dof)
      const int nsimple = neq + nlim + ntr;
      for (int idx = lane + rl0; idx < nsimple * NVW; idx += rls) {
        const int r = idx >> S::LOG_NVW, i = idx & (NVW - 1);
        const int src = s.efc_src[r], kind = src >> 24, id = (src >> 4) & 0xfffff, side = src & 15;
        float v = 0.f;
        if (S::WIDE && kind == 1 && side > 0) {  // connect: (J_p(b1, p1) - J_p(b2, p2))[side - 1]
          const int comp = side - 1;
          if (i < nv) {
            const float* cd = s.cdof[i];
#pragma unroll
            for (int e2 = 0; e2 < 2; e2++) {
              const int bb = e2 == 0 ? m->eq_b1[id] : m->eq_b2[id];
              if (bb >= 0 && ((m->body_dofmask[bb] >> i) & 1u)) {
                const int tr = m->body_tree[bb];
                float r[3] = {s.eqp[id][e2][0] - s.com[tr][0], s.eqp[id][e2][1] - s.com[tr][1],
                              s.eqp[id][e2][2] - s.com[tr][2]}, cr[3];
                cross(cr, cd, r);
                const float jv = cd[3 + comp] + cr[comp];
                v += e2 == 0 ? jv : -jv;
              }
            }
          }
        } else if (kind == 1) {
          const int j1 = m->eq_j1[id], j2 = m->eq_j2[id];
          if (i == m->jnt_dofadr[j1]) v += 1.f;
          if (j2 >= 0 && i == m->jnt_dofadr[j2]) {
            const float* c = m->eq_data[id];
            const float dif = s.qpos[m->jnt_qposadr[j2]] - m->jnt_qpos0[j2];
            v -= c[1] + dif * (2.f * c[2] + dif * (3.f * c[3] + dif * 4.f * c[4]));
          }
        } else if (S::WIDE && kind == 4) {  // tendon: +-(dif / len) . (J_p(site2) - J_p(site1))
          if (i < nv) {
            const float dif[3] = {s.tenp[id][1][0] - s.tenp[id][0][0], s.tenp[id][1][1] - s.tenp[id][0][1],
                                  s.tenp[id][1][2] - s.tenp[id][0][2]};
            const float il = 1.f / fmaxf(sqrtf(dot3(dif, dif)), kMinVal);
            const float* cd = s.cdof[i];
#pragma unroll
            for (int e2 = 0; e2 < 2; e2++) {
              const int bb = m->ten_body[id][e2];
              if (bb >= 0 && ((m->body_dofmask[bb] >> i) & 1u)) {
                const int tr = m->body_tree[bb];
                float rr[3] = {s.tenp[id][e2][0] - s.com[tr][0], s.tenp[id][e2][1] - s.com[tr][1],
                               s.tenp[id][e2][2] - s.com[tr][2]}, cr[3];
                cross(cr, cd, rr);
                const float jp = (dif[0] * (cd[3] + cr[0]) + dif[1] * (cd[4] + cr[1]) + dif[2] * (cd[5] + cr[2])) * il;
                v += e2 == 0 ? -jp : jp;
              }
            }
            if (side) v = -v;
          }
        } else if (i == m->jnt_dofadr[id]) {
          v = side == 0 ? 1.f : -1.f;
        }
        jstore(s, gx, r, i, v);
      }
      // contact Jacobians: (contact, dof) -> J_n +- mu J_t rows
      for (int idx = lane + rl0; idx < keep_con * NVW; idx += rls) {
        const int c = idx >> S::LOG_NVW, i = idx & (NVW - 1);
        const int p = s.con_pair[c];
        const int4 ji = m->pair_jinfo[p];  // one load: both bodies' dof masks and trees
        float jd[3] = {0.f, 0.f, 0.f};
        if (i < nv) {
          const float* cd = s.cdof[i];
#pragma unroll
          for (int side = 0; side < 2; side++) {
            if (((unsigned)(side == 0 ? ji.x : ji.y) >> i) & 1u) {
              const int tr = side == 0 ? ji.z : ji.w;
              float r[3] = {s.con_pos[c][0] - s.com[tr][0], s.con_pos[c][1] - s.com[tr][1],
                            s.con_pos[c][2] - s.com[tr][2]}, cr[3];
              cross(cr, cd, r);
              const float sg = side == 0 ? -1.f : 1.f;
              jd[0] += sg * (cd[3] + cr[0]); jd[1] += sg * (cd[4] + cr[1]); jd[2] += sg * (cd[5] + cr[2]);
            }
          }
        }
        // the contact frame (the wide image keeps only its normal row: the
        // tangents are make_frame's of it, bitwise what emit computed)
        float fw[9];
        const float* f = s.con_frame[c];
        if constexpr (S::FRAMEW == 3) {
          make_frame(fw, s.con_frame[c]);
          f = fw;
        }
        const float jn = f[0] * jd[0] + f[1] * jd[1] + f[2] * jd[2];
        const int off = s.con_row[c];
        if (m->pair_condim[p] == 1) {
          jstore(s, gx, off, i, jn);
        } else if (S::WIDE && m->cone == 1) {  // elliptic: J_n, J_t1, J_t2
          jstore(s, gx, off + 0, i, jn);
          jstore(s, gx, off + 1, i, f[3] * jd[0] + f[4] * jd[1] + f[5] * jd[2]);
          jstore(s, gx, off + 2, i, f[6] * jd[0] + f[7] * jd[1] + f[8] * jd[2]);
        } else {
          const float mu = m->pair_friction[p];
          const float jt1 = f[3] * jd[0] + f[4] * jd[1] + f[5] * jd[2];
          const float jt2 = f[6] * jd[0] + f[7] * jd[1] + f[8] * jd[2];
          jstore(s, gx, off + 0, i, jn + mu * jt1);
          jstore(s, gx, off + 1, i, jn - mu * jt1);
          jstore(s, gx, off + 2, i, jn + mu * jt2);
          jstore(s, gx, off + 3, i, jn - mu * jt2);
        }
      }
      // (also orders the J rows past JL written to the HBM slab by other lanes,
      // and with rows_j the other wave's rows)
      if (rows_j) block_sync();
      else sync();
      // row parameters: vel, impedance, D, aref
      for (int r = lane + rl0; r < nefc; r += rls) {
        const int src = s.efc_src[r], kind = src >> 24, id = (src >> 4) & 0xfffff, side = src & 15;
        float pos, margin, diag;
        const float* sref;
        const float* simp;
        if (S::WIDE && kind == 1 && side > 0) {  // connect component
          pos = s.eqp[id][0][side - 1] - s.eqp[id][1][side - 1];
          margin = 0.f;
          diag = m->eq_diag[id];
          sref = m->eq_solref[id];
          simp = m->eq_solimp[id];
        } else if (kind == 1) {
          const int j1 = m->eq_j1[id], j2 = m->eq_j2[id];
          const float* c = m->eq_data[id];
          const float q1 = s.qpos[m->jnt_qposadr[j1]] - m->jnt_qpos0[j1];
          if (j2 >= 0) {
            const float dif = s.qpos[m->jnt_qposadr[j2]] - m->jnt_qpos0[j2];
            pos = q1 - (c[0] + dif * (c[1] + dif * (c[2] + dif * (c[3] + dif * c[4]))));
          } else {
            pos = q1 - c[0];
          }
          margin = 0.f;
          diag = m->eq_diag[id];
          sref = m->eq_solref[id];
          simp = m->eq_solimp[id];
        } else if (kind == 2) {
          const float q = s.qpos[m->jnt_qposadr[id]];
          pos = side == 0 ? q - m->jnt_range[id][0] : m->jnt_range[id][1] - q;
          margin = m->jnt_margin[id];
          diag = m->dof_invweight0[m->jnt_dofadr[id]];
          sref = m->jnt_solref[id];
          simp = m->jnt_solimp[id];
        } else if (S::WIDE && kind == 4) {
          const float dx = s.tenp[id][1][0] - s.tenp[id][0][0], dy = s.tenp[id][1][1] - s.tenp[id][0][1],
                      dz = s.tenp[id][1][2] - s.tenp[id][0][2];
          const float len = sqrtf(dx * dx + dy * dy + dz * dz);
          pos = side == 0 ? len - m->ten_range[id][0] : m->ten_range[id][1] - len;
          margin = m->ten_margin[id];
          diag = m->ten_invw[id];
          sref = m->ten_solref[id];
          simp = m->ten_solimp[id];
        } else if (S::WIDE && kind == 5) {  // elliptic: all rows take the normal's impedance
          const int c = (src >> 14) & 1023, p = ell_pair(src);
          pos = s.con_dist[c];
          margin = m->pair_margin[p];
          diag = m->pair_diag[p];
          sref = m->pair_solref[p];
          simp = m->pair_solimp[p];
        } else {
          const int p = s.con_pair[id];
          pos = s.con_dist[id];
          margin = m->pair_margin[p];
          const float mu = m->pair_friction[p];
          diag = m->pair_condim[p] == 1 ? m->pair_diag[p] : m->pair_diag[p] * (1.f + mu * mu);
          sref = m->pair_solref[p];
          simp = m->pair_solimp[p];
        }
        const float vel = jdot(s, gx, r, s.qvel);
        const float imp = impedance(simp, pos, margin);
        float R = fmaxf((1.f - imp) / imp * diag, kMinVal);
        // elliptic friction rows: R_t = R_n / impratio (equal sliding
        // frictions), no position term in aref
        const bool efric = S::WIDE && kind == 5 && side > 0;
        if (efric) R = R / m->impratio;
        float tc = sref[0];
        const float dr = sref[1];
        const float dmax = clampf(simp[1], kMinImp, kMaxImp);
        float K, B;
        if (tc > 0.f) {
          if (!(m->disableflags & 2)) tc = fmaxf(tc, 2.f * m->timestep);
          K = 1.f / (dmax * dmax * tc * tc * dr * dr);
          B = 2.f / (dmax * tc);
        } else {
          K = -tc / (dmax * dmax);
          B = -dr / dmax;
        }
        s.efc_D[r] = 1.f / R;
        s.efc_aref[r] = -B * vel - K * imp * (efric ? 0.f : pos - margin);
        if (args.dbg && b == 0 && t == H - 1 && r < DBG_MAXROW) {
          float* o = args.dbg + DBG_ROW + 3 * r;
          o[0] = s.efc_D[r]; o[1] = s.efc_aref[r]; o[2] = vel;
        }
      }
      if (args.dbg && b == 0 && t == H - 1 && run_main) {
        if (lane == 0) { args.dbg[DBG_NCON] = (float)s.ncon; args.dbg[DBG_NEFC] = (float)s.nefc; }
        if (lane < s.ncon && lane < DBG_MAXCON) {
          float* o = args.dbg + DBG_CON + 8 * lane;
          o[0] = s.con_pos[lane][0]; o[1] = s.con_pos[lane][1]; o[2] = s.con_pos[lane][2];
          o[3] = s.con_dist[lane]; o[4] = (float)s.con_pair[lane];
          o[5] = s.con_frame[lane][0]; o[6] = s.con_frame[lane][1]; o[7] = s.con_frame[lane][2];
        }
      }
      sync();
    }  // constraint rows
    if constexpr (WPC == 2) {
      if (rows_j) {
        block_sync();  // the rows are ready
        if (!run_main) {
          // wave 1: each Newton iteration's Hessian (two barriers per
          // iteration, the same count as wave 0's loop), then it waits for
          // the next step's geom poses
          STAMP(8);
          const int nefc = s.nefc;
          // the implicit factor: in the first iteration's wait (wave 0's
          // solve, line search and next active set), else after the loop
          bool fdone = !impl2;
          auto impl_factor = [&]() {
            const float dt = m->timestep;
            float fa[BLK_N], fdinv;
            blocked_factor<BLK_N>(m, [&](int i, int j) { return fmaf(dt, m->impl_D[i][j], m_get(i, j)); }, lane, fa,
                                  fdinv);
#pragma unroll
            for (int j = 0; j < BLK_N; j++) implf[j * WAVE + lane] = fa[j];
            implf[BLK_N * WAVE + lane] = fdinv;
            fdone = true;
          };
          if (hess2 && nefc > 0)
            for (int it = 0; it < m->iterations; it++) {
              block_sync();  // wave 0: efc_Da / efc_jar of this iteration
              STAMP(29);
              newton_hessian(nefc, &s.gxpos[0][0]);
              STAMP(31);
              block_sync();  // wave 0: gradient and stop test
              STAMP(30);
              if (s.pad_) break;
              if (!fdone) impl_factor();
            }
          if (!fdone) impl_factor();
          if (impl2) block_sync();  // the implicit factor, to wave 0's solve
          continue;
        }
      }
      if (rows_c) {
        if (run_coll && lane == 0) s.pad_ = coupled ? 1 : 0;
        block_sync();  // contacts and constraint rows ready; wave 1 waits for the next step's geom poses
        if (!run_main) continue;
        coupled = s.pad_ != 0;
      }
    }
    if (args.dbg && b == 0 && t == H - 1 && lane < NVW) args.dbg[DBG_QAS + lane] = s.qas[lane];
    nefc_sum += s.nefc;
    nefc_max = max(nefc_max, s.nefc);

    STAMP(8);
    STOP_AT(8)
#if MPCR_PACE && MPCR_PACE_AT == 2
    PACE_SETPRIO();
#endif
    LAUNDER_PHASE();  // phase boundary: no cross-phase model-load CSE
    // ---- Newton solver (primal), MJX-style line search ------------------------
    {
      const int nefc = s.nefc;
      float qacc_l = lane < NVW ? s.qas[lane] : 0.f;  // this lane's dof value
      if (nefc > 0) {
        // warm start: the better of qacc_warmstart and qacc_smooth
        if (!(m->disableflags & 4)) {
          // (the Gauss term of qacc_smooth itself is (M a_s - f_s)'(a_s - a_s) = 0)
          const float maw = lane < nv ? m_dot(lane, s.qws) : 0.f;
          const float gw = lane < nv ? (maw - s.qfs[lane]) * (s.qws[lane] - s.qas[lane]) : 0.f;
          float cw = 0.f, cs = 0.f;
          for (int r = lane; r < nefc; r += S::HL) {
            const float jw = jdot(s, gx, r, s.qws) - s.efc_aref[r];
            const float js = jdot(s, gx, r, s.qas) - s.efc_aref[r];
            const bool eq = (s.efc_src[r] >> 24) == 1;
            if constexpr (S::WIDE) {
              if (ell_row(s.efc_src[r])) {
                if (ell_head(s.efc_src[r])) {  // the cone cost of the whole contact
                  const int p = ell_pair(s.efc_src[r]);
                  const float D[3] = {s.efc_D[r], s.efc_D[r + 1], s.efc_D[r + 2]};
                  float xw[3] = {jw, 0.f, 0.f}, xs[3] = {js, 0.f, 0.f}, f[3], h[6];
#pragma unroll
                  for (int k = 1; k < 3; k++) {
                    xw[k] = jdot(s, gx, r + k, s.qws) - s.efc_aref[r + k];
                    xs[k] = jdot(s, gx, r + k, s.qas) - s.efc_aref[r + k];
                  }
                  cw += 2.f * cone_update(xw, m->pair_cmu[p], m->pair_friction[p], D, f, h);
                  cs += 2.f * cone_update(xs, m->pair_cmu[p], m->pair_friction[p], D, f, h);
                }
                continue;
              }
            }
            if (eq || jw < 0.f) cw += s.efc_D[r] * jw * jw;
            if (eq || js < 0.f) cs += s.efc_D[r] * js * js;
          }
          const float costw = 0.5f * hsum<S::CPW>(gw) + 0.5f * hsum<S::CPW>(cw);
          const float costs = 0.5f * hsum<S::CPW>(cs);
          if (costw < costs && lane < NVW) qacc_l = s.qws[lane];
          if (args.dbg && b == 0 && t == H - 1 && lane == 0) {
            args.dbg[DBG_INFO + 0] = costw < costs ? 1.f : 0.f;
            args.dbg[DBG_INFO + 1] = costw;
            args.dbg[DBG_INFO + 2] = costs;
          }
        }
        if (lane < NVW) s.qacc[lane] = qacc_l;
        sync();
        STAMP(13);
        STOP_AT(13)
        const float scale = 1.f / (m->meaninertia * (float)(nv > 1 ? nv : 1));
        float prev_cost = 3.4e38f;
        for (int it = 0;; it++) {
          // the iteration cap ends the solve before anything below matters
          // (cost / gradient only feed the stop test)
          if (it >= m->iterations) break;
#ifdef MPCR_PROFILE
          prof_acc[15] += 1;  // Newton iterations (low half of the counter, not cycles)
#endif
#ifdef MPCR_WAVETIME
          wt_newton++;
#endif
          // Ma, jar, cost at the current qacc; per-row force and active D
          const float ma = lane < nv ? m_dot(lane, s.qacc) : 0.f;
          float cc = 0.f;
          for (int r = lane; r < nefc; r += S::HL) {
            const float jar = jdot(s, gx, r, s.qacc) - s.efc_aref[r];
            bool act = ((s.efc_src[r] >> 24) == 1) || jar < 0.f;
            if constexpr (S::WIDE) act = act && !ell_row(s.efc_src[r]);  // cone pass below
            const float D = s.efc_D[r];
            s.efc_jar[r] = jar;
            s.efc_f[r] = act ? -D * jar : 0.f;
            s.efc_Da[r] = act ? D : 0.f;
            cc += act ? D * jar * jar : 0.f;
          }
          if constexpr (S::WIDE) {  // elliptic contacts: cone cost and forces
            if (m->cone == 1) {
              sync();
              for (int r = lane; r < nefc; r += S::HL) {
                const int src = s.efc_src[r];
                if (!ell_head(src)) continue;
                const int p = ell_pair(src);
                const float x[3] = {s.efc_jar[r], s.efc_jar[r + 1], s.efc_jar[r + 2]};
                const float D[3] = {s.efc_D[r], s.efc_D[r + 1], s.efc_D[r + 2]};
                float f[3], h[6];
                cc += 2.f * cone_update(x, m->pair_cmu[p], m->pair_friction[p], D, f, h);
                s.efc_f[r] = f[0]; s.efc_f[r + 1] = f[1]; s.efc_f[r + 2] = f[2];
              }
            }
          }
          const float gauss = hsum<S::CPW>(lane < nv ? (ma - s.qfs[lane]) * (s.qacc[lane] - s.qas[lane]) : 0.f);
          const float cost = 0.5f * gauss + 0.5f * hsum<S::CPW>(cc);
          sync();
          if (hess2) block_sync();  // this iteration's active set, to wave 1
          STAMP(29);
          constexpr bool MFMA_HESS = NVW == 16 && S::CPW == 1 && MPCR_MFMA_HESS;
          constexpr bool MFMA_HESS_W = NVW == 32 && S::CPW == 1 && MPCR_MFMA_HESS_W;
          constexpr int RPW = S::HL / NVW;
          const int gi = lane & (NVW - 1), gq = lane >> S::LOG_NVW;
          float* Hs = &s.gxpos[0][0];  // geom poses are dead during Newton
          float grad;
          if constexpr (MFMA_HESS) {
            // J^T f and H = M + J^T D_active J together on the matrix core,
            // 4 rows per v_mfma_f32_16x16x4_f32: lane (dof gi, row r0 + gq)
            // supplies A = J[r][gi] and B = D_a J[r][gi] (Hessian) / f[r]
            // (gradient); accumulator register v of lane l is column gi of
            // row 4 gq + v -- read as row gi of H that is the float4
            // H[gi][4 gq ..], the same products in the same row order as the
            // VALU build (the MFMA is a k-ordered fmaf chain), so H is
            // bitwise the VALU one
            const float4 m4 = m_quad(gi, gq);
            mfx4 hacc = {m4.x, m4.y, m4.z, m4.w};
            mfx4 gacc = {0.f, 0.f, 0.f, 0.f};
            for (int r0 = 0; r0 < nefc; r0 += 4) {
              const int r = r0 + gq;
              const bool ok = r < nefc;
              const float a = ok ? jrow_ptr(s, gx, r)[gi] : 0.f;
              const float da = ok ? s.efc_Da[r] : 0.f;
              const float fr = ok ? s.efc_f[r] : 0.f;
              hacc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, da * a, hacc, 0, 0, 0);
              gacc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, fr, gacc, 0, 0, 0);
            }
            reinterpret_cast<float4*>(Hs + gi * S::LD)[gq] = make_float4(hacc[0], hacc[1], hacc[2], hacc[3]);
            float* qcs = Hs + NVW * S::LD;  // J^T f: lanes 0, 16, 32, 48 hold dofs 4 gq ..
            if (gi == 0) reinterpret_cast<float4*>(qcs)[gq] = make_float4(gacc[0], gacc[1], gacc[2], gacc[3]);
            sync();
            grad = lane < nv ? ma - s.qfs[lane] - qcs[gi] : 0.f;
          } else if constexpr (MFMA_HESS_W) {
            // 32-wide: J^T f on v_mfma_f32_32x32x2_f32, 2 rows per instruction
            // (lane: A = J[r0 + gq][gi], B = f[r0 + gq]); accumulator register
            // v of lane l holds (J^T f)[(v & 3) + 8 (v >> 2) + 4 gq]
            mfx16 gacc;
#pragma unroll
            for (int v = 0; v < 16; v++) gacc[v] = 0.f;
            gacc = mfma_rows32(s, gx, nefc, gi, gq, [&](int r, float) { return s.efc_f[r]; }, gacc);
            float* qcs = s.srch;  // free until this iteration's search direction
            if (gi == 0) {
#pragma unroll
              for (int k = 0; k < 4; k++)
                reinterpret_cast<float4*>(qcs + 8 * k + 4 * gq)[0] =
                    make_float4(gacc[4 * k], gacc[4 * k + 1], gacc[4 * k + 2], gacc[4 * k + 3]);
            }
            sync();
            grad = lane < nv ? ma - s.qfs[lane] - qcs[gi] : 0.f;
            sync();  // qcs (srch) is rewritten below
          } else {
            // grad = Ma - qfrc_smooth - J^T f: lane (dof i, row group q); RPW
            // lanes share a dof (4 at NVW 16, 2 at NVW 32)
            float qc = 0.f;
            jrows(s, gx, gq, RPW, nefc, [&](const float* J, int r) { qc = fmaf(J[gi], s.efc_f[r], qc); });
#pragma unroll
            for (int o = NVW; o < S::HL; o <<= 1) qc += __shfl_xor(qc, o);
            grad = lane < nv ? ma - s.qfs[lane] - qc : 0.f;
          }
          STAMP(30);
          const float gn = sqrtf(hsum<S::CPW>(grad * grad));
          // MuJoCo's stop test, plus its fp32 floor: an improvement within ~8 ulp
          // of the cost is rounding noise (without it fp32 iterates on noise
          // where the fp64 solve has converged: 3.9 vs 1.9 iterations per
          // dual-arm step)
          const bool stop = scale * (prev_cost - cost) < m->tolerance || scale * gn < m->tolerance ||
                            prev_cost - cost <= 1e-6f * fabsf(cost);
          if (hess2) {  // hand the decision to wave 1, take its Hessian
            if (lane == 0) s.pad_ = stop ? 1 : 0;
            block_sync();
          }
          if (stop) break;
          if constexpr (!MFMA_HESS) {
            if (!hess2) newton_hessian(nefc, Hs);  // (two waves: wave 1 built it meanwhile)
          }
          STAMP(31);
          float mg;
          if (S::CPW == 1 && !coupled && blk_usable<NVW>(m)) {
            // no row couples two trees: H is block diagonal like M
            if (lane < NVW) s.srch[lane] = lane < nv ? grad : 0.f;
            sync();
            blk_solve<NVW>(m, [&](int i, int j) { return Hs[i * S::LD + j]; }, s.srch, s.srch, lane, &s.gxpos[0][0]);
            sync();
            mg = lane < nv ? s.srch[lane] : 0.f;
            sync();  // srch is rewritten below
          } else {
            float h[NVW];
            {
              const float4* row = reinterpret_cast<const float4*>(Hs + (lane & (NVW - 1)) * S::LD);
#pragma unroll
              for (int q = 0; q < NVW / 4; q++) {
                const float4 v = row[q];
                h[4 * q] = v.x; h[4 * q + 1] = v.y; h[4 * q + 2] = v.z; h[4 * q + 3] = v.w;
              }
            }
            if constexpr (NVW == 16 && MPCR_DPP_CHOL) {
              float dinv;
              chol16(h, dinv, lane);
              mg = chol16_solve<S::LD>(h, dinv, lane < nv ? grad : 0.f, lane, &s.gxpos[0][0]);
            } else {
              chol_rows(h, lane);
              mg = chol_solve<NVW, S::LD>(h, lane < nv ? grad : 0.f, lane, &s.gxpos[0][0]);
            }
          }
          const float search = lane < nv ? -mg : 0.f;
          if (args.dbg && b == 0 && t == H - 1 && it == 0 && lane < NVW) {
            args.dbg[DBG_GRAD + lane] = grad;
            args.dbg[DBG_SRCH + lane] = search;
          }
          STAMP(14);
          if (lane < NVW) s.srch[lane] = search;
          sync();
          // Mv, jv, quadratic coefficients
          const float mvv = lane < nv ? m_dot(lane, s.srch) : 0.f;
          for (int r = lane; r < nefc; r += S::HL) s.efc_jv[r] = jdot(s, gx, r, s.srch);
          const float sn = sqrtf(hsum<S::CPW>(search * search));
          const float gtol = m->tolerance * m->ls_tolerance * sn * m->meaninertia * (float)(nv > 1 ? nv : 1);
          float qg[3];
          qg[0] = 0.5f * gauss;
          qg[1] = hsum<S::CPW>(lane < nv ? search * (ma - s.qfs[lane]) : 0.f);
          qg[2] = 0.5f * hsum<S::CPW>(search * mvv);
          sync();
          using LT = LsReal<S>;
          using LsPt = LsPtT<LT>;
          LsPt p0 = ls_eval(s, lane, qg, (LT)0);
          const bool ell_ls = S::WIDE && m->cone == 1;
          if (ell_ls) {
            const LT al[3] = {0, 0, 0};
            float e[9];
            ls_cones3(s, m, lane, al, e);
            ls_add(p0, e[0], e[1], e[2]);
          }
          constexpr bool LSQ0 = S::WIDE;  // narrow: q0 deferred to ls_finish
          LsPt lo = ls_eval<S, LSQ0>(s, lane, qg, p0.alpha - p0.d0 / p0.d1);
          if (ell_ls) {
            const LT al[3] = {lo.alpha, 0, 0};
            float e[9];
            ls_cones3(s, m, lane, al, e);
            ls_add(lo, e[0], e[1], e[2]);
          }
          LsPt hi;
          if (lo.d0 < p0.d0) { hi = p0; } else { hi = lo; lo = p0; }
          bool swap = true;
          for (int ls = 0; ls < m->ls_iterations; ls++) {
            if (!swap) break;
#ifdef MPCR_PROFILE
            prof_acc[15] += 1ull << 32;  // line-search passes (high half of the counter)
#endif
#ifdef MPCR_WAVETIME
            wt_ls++;
#endif
            if (args.dbg && b == 0 && t == H - 1 && lane == 0 && it == 0) args.dbg[DBG_INFO + 5] = (float)ls;
            if (lo.d0 < 0.f && lo.d0 > -gtol) break;
            if (hi.d0 > 0.f && hi.d0 < gtol) break;
            // bracket closed to fp32 resolution: further passes only move alpha
            // by rounding noise (gtol sits below fp32 resolution; without this the
            // dual arm ran ~20 passes per Newton iteration against ~2.4 in fp64)
            {
              const LT da = hi.alpha - lo.alpha, la = lo.alpha < 0 ? -lo.alpha : lo.alpha,
                       ha = hi.alpha < 0 ? -hi.alpha : hi.alpha;
              if ((da < 0 ? -da : da) <= (LT)1e-6f * (la > ha ? la : ha)) break;
            }
            LsPt lo_next, hi_next, mid;
            ls_eval3<S, LSQ0>(s, lane, qg, lo.alpha - lo.d0 / lo.d1, hi.alpha - hi.d0 / hi.d1,
                              (LT)0.5 * (lo.alpha + hi.alpha), lo_next, hi_next, mid);
            if (ell_ls) {
              const LT al[3] = {lo_next.alpha, hi_next.alpha, mid.alpha};
              float e[9];
              ls_cones3(s, m, lane, al, e);
              ls_add(lo_next, e[0], e[1], e[2]);
              ls_add(hi_next, e[3], e[4], e[5]);
              ls_add(mid, e[6], e[7], e[8]);
            }
            const bool s1 = lo.d0 > 0.f || lo.d0 < lo_next.d0;
            if (s1) lo = lo_next;
            const bool s2 = mid.d0 < 0.f && lo.d0 < mid.d0;
            if (s2) lo = mid;
            const bool s3 = hi.d0 < 0.f || hi.d0 > hi_next.d0;
            if (s3) hi = hi_next;
            const bool s4 = mid.d0 > 0.f && hi.d0 > mid.d0;
            if (s4) hi = mid;
            swap = s1 || s2 || s3 || s4;
          }
          if constexpr (!LSQ0) ls_finish(s, lane, qg, lo, hi);
          const bool improved = lo.cost < p0.cost || hi.cost < p0.cost;
          const LT alpha = lo.cost < hi.cost ? lo.alpha : hi.alpha;
          if (args.dbg && b == 0 && t == H - 1 && lane == 0 && it == 0) {
            args.dbg[DBG_INFO + 3] = (float)p0.cost;
            args.dbg[DBG_INFO + 4] = (float)alpha;
            args.dbg[DBG_INFO + 6] = (float)(lo.cost < hi.cost ? lo.cost : hi.cost);
          }
          if (args.dbg && b == 0 && t == H - 1 && lane == 0) args.dbg[DBG_INFO + 7] = (float)(it + 1);
          if (improved && lane < NVW) s.qacc[lane] = (float)((LT)s.qacc[lane] + alpha * (LT)s.srch[lane]);
          prev_cost = cost;
          sync();
          STAMP(9);
        }
      } else {
        if (lane < NVW) s.qacc[lane] = qacc_l;
        sync();
      }
    }

    if (args.dbg && b == 0 && t == H - 1 && lane < NVW) args.dbg[DBG_QACC + lane] = s.qacc[lane];
    STAMP(9);
    STOP_AT(9)
    LAUNDER_PHASE();  // phase boundary: no cross-phase model-load CSE
    // ---- implicitfast (dual-arm class): (M + dt D) a = qfrc_smooth + J^T f at
    //      the final qacc; the velocity update uses a, the warm start qacc --
    bool implicit = false;
    if constexpr (S::WIDE) {
      if (m->integrator == 3) {
        implicit = true;
        const int nefc = s.nefc;
        for (int r = lane; r < nefc; r += S::HL) {
          const float jar = jdot(s, gx, r, s.qacc) - s.efc_aref[r];
          const bool act = ((s.efc_src[r] >> 24) == 1) || jar < 0.f;
          s.efc_f[r] = act ? -s.efc_D[r] * jar : 0.f;
          s.efc_jar[r] = jar;
        }
        sync();
        if (m->cone == 1) {  // elliptic contacts: cone forces at the final qacc
          for (int r = lane; r < nefc; r += S::HL) {
            const int src = s.efc_src[r];
            if (!ell_head(src)) continue;
            const int p = ell_pair(src);
            const float x[3] = {s.efc_jar[r], s.efc_jar[r + 1], s.efc_jar[r + 2]};
            const float D[3] = {s.efc_D[r], s.efc_D[r + 1], s.efc_D[r + 2]};
            float f[3], h[6];
            cone_update(x, m->pair_cmu[p], m->pair_friction[p], D, f, h);
            s.efc_f[r] = f[0]; s.efc_f[r + 1] = f[1]; s.efc_f[r + 2] = f[2];
          }
          sync();
        }
        constexpr int RPW = S::HL / NVW;
        const int gi = lane & (NVW - 1), gq = lane >> S::LOG_NVW;
        float qc = 0.f;
        jrows(s, gx, gq, RPW, nefc, [&](const float* J, int r) { qc = fmaf(J[gi], s.efc_f[r], qc); });
#pragma unroll
        for (int o = NVW; o < S::HL; o <<= 1) qc += __shfl_xor(qc, o);
        const float dt = m->timestep;
        if (S::CPW == 1 && !m->impl_cross && blk_usable<NVW>(m)) {  // M + dt D block diagonal by tree
          if (lane < NVW) s.srch[lane] = lane < nv ? s.qfs[lane] + qc : 0.f;
          sync();
          if (impl2) {  // wave 1's factor
            block_sync();
            float fa[BLK_N];
#pragma unroll
            for (int j = 0; j < BLK_N; j++) fa[j] = implf[j * WAVE + lane];
            blocked_sweep<BLK_N>(m, fa, implf[BLK_N * WAVE + lane], s.srch, s.srch, lane, &s.gxpos[0][0]);
          } else {
            blk_solve<NVW>(m, [&](int i, int j) { return fmaf(dt, m->impl_D[i][j], m_get(i, j)); }, s.srch, s.srch,
                           lane, &s.gxpos[0][0]);
          }
          sync();
        } else {
          float Lm[NVW];
#pragma unroll
          for (int j = 0; j < NVW; j++) Lm[j] = lane < NVW ? fmaf(dt, m->impl_D[lane][j], m_get(lane, j)) : 0.f;
          chol_rows(Lm, lane);
          const float a = chol_solve<NVW, S::LD>(Lm, lane < nv ? s.qfs[lane] + qc : 0.f, lane, &s.gxpos[0][0]);
          if (lane < NVW) s.srch[lane] = lane < nv ? a : 0.f;
          sync();
        }
      }
    }
    // ---- Euler: qvel += dt qacc; integrate qpos; warm start -----------------
    {
      const float dt = m->timestep;
      if (lane < nv) {
        s.qvel[lane] = s.qvel[lane] + dt * (implicit ? s.srch[lane] : s.qacc[lane]);
        s.qws[lane] = s.qacc[lane];
      }
      sync();
      if (lane < m->njnt) {
        const int a = m->jnt_qposadr[lane], v = m->jnt_dofadr[lane], type = m->jnt_type[lane];
        if (type == 0) {
          s.qpos[a] += dt * s.qvel[v];
          s.qpos[a + 1] += dt * s.qvel[v + 1];
          s.qpos[a + 2] += dt * s.qvel[v + 2];
          float w[3] = {s.qvel[v + 3], s.qvel[v + 4], s.qvel[v + 5]};
          float q[4] = {s.qpos[a + 3], s.qpos[a + 4], s.qpos[a + 5], s.qpos[a + 6]};
          const float wn = sqrtf(dot3(w, w));
          const float ang = wn * dt;
          if (ang > kMinVal) {
            float sn, cs;
            __sincosf(0.5f * ang, &sn, &cs);
            float dq[4] = {cs, w[0] / wn * sn, w[1] / wn * sn, w[2] / wn * sn};
            qmul(q, q, dq);
          }
          float n = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
          s.qpos[a + 3] = q[0] / n; s.qpos[a + 4] = q[1] / n; s.qpos[a + 5] = q[2] / n; s.qpos[a + 6] = q[3] / n;
        } else if (type == 2 || type == 3) {
          s.qpos[a] += dt * s.qvel[v];
        }
      }
      sync();
      if (lane < nc && args.theta && live) args.theta[(size_t)b * nc * H + lane * H + t] = s.qpos[ctrl_qa];
    }
  }

  STAMP(10);
  PROF_FLUSH
  if (args.plant && live && run_main) {  // single-environment plant: qacc of the last step, state back
    if (lane < nv) args.state[ST_QACC + lane] = s.qacc[lane];
    if (args.plant & 2) {
      if (lane < m->nq) args.state[ST_QPOS + lane] = s.qpos[lane];
      if (lane < nv) {
        args.state[ST_QVEL + lane] = s.qvel[lane];
        args.state[ST_QWS + lane] = s.qws[lane];
      }
    }
  }
  if (suspend) {  // not the last segment: save the state and the accumulators, no outputs
    for (int i = lane; i < DX_NQ; i += S::HL) segs[SEG_QPOS + i] = i < S::NQW ? s.qpos[i] : 0.f;
    if (lane < NVW) {
      segs[SEG_QVEL + lane] = s.qvel[lane];
      segs[SEG_QWS + lane] = s.qws[lane];
    }
    segs[SEG_COSTC + lane] = cost_c;
    if (lane == 0) {
      float* sc = segs + SEG_SCAL;
      sc[0] = cost_g; sc[1] = cost_r;
      sc[2] = __int_as_float(status); sc[3] = __int_as_float(nefc_sum); sc[4] = __int_as_float(nefc_max);
    }
#if MPCR_PACE
    if (pace && lane == pace_own) __hip_atomic_store(pace + lane, ~0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
    return;
  }
  // ---- final reductions, outputs ----------------------------------------------
  cost_c = hsum<S::CPW>(cost_c);
  if constexpr (WPC == 2) {  // the collision wave's cost_c and truncation flag
    block_sync();  // wave 0's last step is done with the image (srch)
    if (wv == 1 && lane == 0) { s.srch[0] = cost_c; s.pad_ = status; }
    block_sync();
    if (wv == 1) return;
    cost_c = s.srch[0];
    status |= s.pad_;
  }
  bool finite = true;
  if (lane < m->nq) finite = isfinite(s.qpos[lane]);
  finite = hballot<S::CPW>(!finite) == 0;
  if (!finite) status |= 2;
  if (lane == 0 && live) {
    // a lost two-wave handshake (MPCR_STATUS_SYNC) voids the rollout: +inf
    // keeps it out of the argmin and the elites (a NaN would win the argmin)
    const float cost = (status & (1 << 10)) ? __builtin_inff()
                                            : s.par[PAR_W] * cost_g + s.par[PAR_W + 1] * cost_r + s.par[PAR_W + 2] * cost_c;
    args.cost4[4 * (size_t)b + 0] = cost;
    args.cost4[4 * (size_t)b + 1] = cost_g;
    args.cost4[4 * (size_t)b + 2] = cost_r;
    args.cost4[4 * (size_t)b + 3] = cost_c;
    if (args.status) args.status[b] = status | (min(nefc_max, 255) << 2) | (nefc_sum << 11);
    if (args.best_key) {
      const uint32_t u = __float_as_uint(cost);
      uint32_t key = isnan(cost) ? 0u : ((u & 0x80000000u) ? ~u : (u | 0x80000000u));
      const unsigned long long k64 = ((unsigned long long)key << 32) | (uint32_t)(args.index_base + b);
      atomicMin(args.best_key, k64);
    }
  }
#if MPCR_PACE
  if (pace && lane == pace_own) __hip_atomic_store(pace + lane, ~0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
#ifdef MPCR_WAVETIME
  if (lane == 0 && live && args.prof) {
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), t1 = __builtin_amdgcn_s_memrealtime();
    const unsigned hwid = __builtin_amdgcn_s_getreg((31 << 11) | 4), xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    args.prof[4 * (size_t)b + 0] = wt_t0;
    args.prof[4 * (size_t)b + 1] = t1;
    args.prof[4 * (size_t)b + 2] = c1 - wt_c0;
    args.prof[4 * (size_t)b + 3] = ((unsigned long long)xcc << 32) | hwid;
    args.prof[4 * (size_t)args.n + 2 * (size_t)b] = ((unsigned long long)wt_ls << 32) | wt_newton;
    args.prof[4 * (size_t)args.n + 2 * (size_t)b + 1] = wt_cvx;
  }
#endif
}


// ---------------------------------------------------------------------------
// launchers (the host side lives in another translation unit)
//
// This file is compiled twice (manipulator_mujoco_amd/build.py): MPCR_TU = 1
// holds the single-arm kernels and the launch logic, with the fast-math
// device flags (C3 is VALU-bound: 1.60 ms, 1.86 ms without them); MPCR_TU = 2
// holds the dual-arm kernels, compiled without them (IEEE division / square
// root, no reassociation): the latency-bound dual arm pays ~5 % and its fp32
// rollouts stay within the scalar fp32 restatement's drift (C4 shard
// well-conditioned misses 22 -> 8, worst 4.8e-3 -> 7.8e-4).
// MPCR_TU undefined (0): everything in one unit.
#ifndef MPCR_TU
#define MPCR_TU 0
#endif

// Dual-arm batches up to min(this, the narrow threshold below) run two waves
// per candidate too (rollout_kernel<32, 32, 72, true, 2>: collision, the MPR
// flush and the manifolds beside the dynamics).  Its 29 KB image and 235
// VGPRs leave 4 blocks per CU, so the default is 4 x 256 CUs: every candidate
// resident in one round (measured on MI355X, H = 100: 1024 candidates 22.6 ->
// 21.2 ms; 2048 would take two rounds, 24.5 -> 46.3 ms).  Bitwise the one-wave
// results.  MPCR_WPC2W_MAX_N overrides.
#ifndef MPCR_W_WPC2
#define MPCR_W_WPC2 1
#endif
// extra dynamic LDS per one-wave dual-arm block (occupancy experiments only)
#ifndef MPCR_W_DYN_LDS
#define MPCR_W_DYN_LDS 0
#endif

#if MPCR_TU != 1
// the dual-arm kernels' launches (rollout_launch's wide branch calls these)
void rollout_wide_launch(int wpc, unsigned grid, hipStream_t st, const RolloutArgs& a, const DevModel* dm) {
  if (wpc == 2)
    hipLaunchKernelGGL((rollout_kernel<32, 32, 72, true, 2>), dim3(grid), dim3(2 * WAVE), 0, st, a, dm);
  else
    hipLaunchKernelGGL((rollout_kernel<32, 32, 72, true>), dim3(grid), dim3(WAVE), MPCR_W_DYN_LDS, st, a, dm);
}
hipError_t rollout_wide_occupancy(int* info) {
  const void* k = reinterpret_cast<const void*>(&rollout_kernel<32, 32, 72, true>);
  int blocks = 0;
  hipFuncAttributes fa;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k, WAVE, MPCR_W_DYN_LDS);
  if (e != hipSuccess) return e;
  e = hipFuncGetAttributes(&fa, k);
  if (e != hipSuccess) return e;
  info[0] = blocks;
  info[1] = (int)fa.sharedSizeBytes;
  info[2] = fa.numRegs;
  return hipSuccess;
}
#endif

#if MPCR_TU != 2
// batches up to this many candidates run the narrow variant with two waves
// per candidate (MPCR_WPC2_MAX_N overrides; 0 disables): below one
// candidate per SIMD pair the second wave of a SIMD is otherwise idle
// (process-wide, atomic: read by every engine's launches, initialised once
// from the environment when the library loads)
static int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}
static std::atomic<int> g_wpc2_max_n{env_int("MPCR_WPC2_MAX_N", MPCR_WPC2_MAX_N_DEFAULT)};
#ifdef MPCR_STOP_AFTER
// attribution builds stop a wave mid-step; the two-wave kernels would leave
// its partner at an unmatched barrier, so these builds run one wave only
static int wpc2_max_n() { return 0; }
#else
static int wpc2_max_n() { return g_wpc2_max_n.load(std::memory_order_relaxed); }
#endif
int rollout_set_wpc2_max_n(int n) {
  return n >= 0 ? g_wpc2_max_n.exchange(n) : wpc2_max_n();
}
#if MPCR_W_WPC2
static const int g_wpc2w_max_n = env_int("MPCR_WPC2W_MAX_N", 1024);
static int wpc2w_max_n() { return min(g_wpc2w_max_n, wpc2_max_n()); }
#endif

// RolloutArgs of candidates [off, off + n) of a launch: the per-candidate
// pointers advanced by off (the kernel indexes them by its block)
static RolloutArgs group_args(const RolloutArgs& a, int off, int n) {
  RolloutArgs g = a;
  const size_t o = (size_t)off;
  g.n = n;
  g.index_base = a.index_base + off;
  const size_t in_row = a.layout == 0 ? (size_t)a.nctrl * a.nbasis : (size_t)a.nctrl * a.H;
  g.input = a.input + o * in_row;
  g.cost4 = a.cost4 + 4 * o;
  const size_t th_row = (size_t)a.nctrl * a.H;
  if (a.theta) g.theta = a.theta + o * th_row;
  if (a.thetadot) g.thetadot = a.thetadot + o * th_row;
  if (a.status) g.status = a.status + o;
  if (a.trace_eef) g.trace_eef = a.trace_eef + o * a.H * 7;
  if (a.trace_slots) g.trace_slots = a.trace_slots + o * a.H * a.nslot;
  g.jx = a.jx + o * (SmemW::MAXEFC - SmemW::JL) * SmemW::LDJ;
  g.hints = a.hints + o * SmemW::NHINT * 2;
  g.mslab = a.mslab + o * SmemW::NVW * SmemW::LD;
  g.tdscratch = a.tdscratch + o * th_row;
  g.slot_prev = a.slot_prev + o * (a.nslot > 0 ? a.nslot : 1);
  g.seg_state = a.seg_state + o * SEG_STRIDE;
  return g;
}

// whether rollout_launch runs a batch as horizon segments, and over how many
// candidate groups (*G)
static bool seg_plan(bool wide, const RolloutArgs& a, unsigned grid, int groups, bool streams, int* G) {
  if (!wide) return false;
#if MPCR_W_WPC2
  if ((int)grid <= wpc2w_max_n()) return false;
#endif
  if (!(a.seg > 0 && a.seg < a.H && a.seg_state && !a.plant && !a.dbg && (int)grid > a.seg_min_n)) return false;
  *G = groups > 1 && streams && (int)grid >= 2 * groups ? groups : 1;
  return true;
}

int rollout_dispatches(bool wide, const RolloutArgs& a, unsigned grid, int groups, bool streams) {
  int G = 1;
  if (grid == 0) return 0;
  if (!seg_plan(wide, a, grid, groups, streams, &G)) return 1;
  return G * ((a.H + a.seg - 1) / a.seg);
}

void rollout_launch(bool wide, const RolloutArgs& a0, const DevModel* dm, unsigned grid, size_t dyn_lds,
                    hipStream_t st, int groups, hipStream_t* gstream, hipEvent_t* gev) {
  RolloutArgs a = a0;
  a.t0 = 0;
  a.t1 = a.H;
  int G = 1;
#if MPCR_W_WPC2
  if (wide && (int)grid <= wpc2w_max_n())
    rollout_wide_launch(2, grid, st, a, dm);
  else
#endif
  if (wide) {
    if (seg_plan(wide, a, grid, groups, gstream && gev, &G)) {
      // horizon segments over candidate groups on their own streams: each
      // group's segments in its stream's order, the groups overlapping
      if (G > 1) {
        (void)hipEventRecord(gev[0], st);
        for (int g = 0; g < G; g++) (void)hipStreamWaitEvent(gstream[g], gev[0], 0);
      }
      const int per = ((int)grid + G - 1) / G;
      for (int g = 0; g < G; g++) {
        const int off = g * per, ng = min(per, (int)grid - off);
        if (ng <= 0) break;
        RolloutArgs ga = G > 1 ? group_args(a, off, ng) : a;
        hipStream_t gs = G > 1 ? gstream[g] : st;
        for (int t0 = 0; t0 < a.H; t0 += a.seg) {
          ga.t0 = t0;
          ga.t1 = min(a.H, t0 + a.seg);
          rollout_wide_launch(1, ng, gs, ga, dm);
        }
      }
      if (G > 1)
        for (int g = 0; g < G; g++) {
          (void)hipEventRecord(gev[1 + g], gstream[g]);
          (void)hipStreamWaitEvent(st, gev[1 + g], 0);
        }
    } else {
      rollout_wide_launch(1, grid, st, a, dm);
    }
  } else {
    if constexpr (SmemN::CPW == 1) {
      if ((int)grid <= wpc2_max_n()) {
        hipLaunchKernelGGL((rollout_kernel<16, 16, 24, false, 2>), dim3(grid), dim3(2 * WAVE), 0, st, a, dm);
        return;
      }
    }
    hipLaunchKernelGGL((rollout_kernel<16, 16, 24, false>), dim3((grid + SmemN::CPW - 1) / SmemN::CPW), dim3(WAVE),
                       dyn_lds, st, a, dm);
  }
}

hipError_t rollout_occupancy(int* info, size_t dyn_lds) {
  const void* k = reinterpret_cast<const void*>(&rollout_kernel<16, 16, 24, false>);
  int blocks = 0;
  hipFuncAttributes fa;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k, WAVE, dyn_lds);
  if (e != hipSuccess) return e;
  e = hipFuncGetAttributes(&fa, k);
  if (e != hipSuccess) return e;
  info[0] = blocks;
  info[1] = (int)fa.sharedSizeBytes;
  info[2] = fa.numRegs;
  return rollout_wide_occupancy(info + 3);
}
#endif  // MPCR_TU != 2

}  // namespace mpcr
