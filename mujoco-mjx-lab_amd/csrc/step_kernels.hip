// mjx355 physics kernels for gfx950 (MI355X / CDNA4).
//
// One 64-lane wavefront (= one 64-thread workgroup) owns one environment for the whole step:
// every stage of mjx.step (reference src/envs.py:345; upstream mujoco-mjx 3.3.6) runs inside a
// single launch with per-env scratch in LDS, so state crosses HBM once per step (read qpos/qvel/
// qacc_warmstart/ctrl/aux, write them back plus obs/reward/done). Inside the wave the work is
// spread over lanes by the natural parallel axis of each stage:
//   kinematics / com_vel+rne forward pass  lane = body, tree levels serialised   (smooth.py)
//   subtree sums (com, crb, rne backward)  lane = body, DFS-contiguous ranges    (smooth.py)
//   cdof, mass-matrix columns, tendons     lane = dof / tendon                   (smooth.py)
//   collision                              lane = candidate geom pair            (collision_*.py)
//   constraint rows (J, D, aref)           lane = dof (J entries) / row (params) (constraint.py)
//   Newton: H = M + J'DJ                   lane = (column, half of rows of H)    (solver.py)
//           Cholesky / triangular solves   lane = matrix row in VGPRs, v_readlane broadcasts
//           exact line search              lane = constraint row + DPP wave reductions
//   integrate                              lane = dof / joint                    (forward.py)
//   env reward / obs / reset               lane 0 scalars + lane = obs entry     (src/envs.py)
// Divergence between envs costs nothing: each wave runs its own number of Newton / line-search
// iterations (unlike vmap's lockstep while_loop).
//
// Code layout: every stage is a __noinline__ function taking address-space-qualified pointers
// (LDS workspace, constant-memory model), so each routine exists once in the code object and the
// hot loop (H build, factor, solve, line search) stays resident in the instruction cache.
#include <hip/hip_runtime.h>

#include "model_dev.h"

namespace mjl {

#define LDSA __attribute__((address_space(3)))
#define CSTA __attribute__((address_space(4)))
#define GLBA __attribute__((address_space(1)))
#define NOINL __device__ __noinline__
// The hot phases are inlined into the kernel entry: a kernel has no callee-saved registers, while a
// called phase function saves every callee-saved VGPR block it touches (v40-47, v56-63, ...) to
// scratch on entry; at 130-250 VGPRs per phase that was ~35 KB of scratch traffic per env-step.
#ifndef MJL_NOINLINE_PHASES
#define PHASE __device__ __forceinline__
#else
#define PHASE NOINL
#endif
#define INL __device__ __forceinline__
#define SYNC() __syncthreads()

// XCD-aware env order. The dispatcher deals workgroups round-robin over the 8 XCDs (MI355X_MICROARCH.md,
// workgroup dispatch: observed, speed only), so with env = blockIdx.x the neighbours of an env -- whose
// 108-112-B segments of every per-env array (qpos, qvel, qacc_warmstart, ctrl, aux, obs ...) share its
// 128-B lines -- run on the other seven XCDs, and each line is fetched and written back through up to
// three L2s. Block b = 8k + x (XCD slot x) runs env (8 (k / C) + x) C + k % C: runs of C = 16 consecutive
// envs on one XCD, the runs dealt round-robin over the XCDs so each XCD still holds envs from the whole
// batch (a contiguous eighth per XCD, which puts e.g. the speed test's highest initial velocities on one
// XCD, measured 0.4-0.6 % slower). Blocks past the last whole round of 8 C keep env = b. Results do not
// depend on the order. Measured (2048 envs, profiles/r5/env_order_ab.json): HBM bytes per launch pooled env
// step 5.78 -> 3.93 MB, in place 6.88 -> 5.05 MB, speed test 1.37 -> 1.15 MB; kernel times unchanged.
INL int block_env() {
  constexpr int C = 16;
  const int b = blockIdx.x, n = gridDim.x;
#ifdef MJL_BLOCK_ORDER  // A/B builds only: env = blockIdx.x
  return b;
#endif
  if (b >= n / (8 * C) * (8 * C)) return b;
  const int x = b & 7, k = b >> 3;
  return ((k / C) * 8 + x) * C + (k % C);
}

#ifdef MJL_TIMING  // diagnostic build only: per-phase s_memtime stamps to a side buffer
__device__ unsigned long long* g_stamps;
#define STAMP(slot, lane)                                                                        \
  do {                                                                                           \
    unsigned long long t_ = __builtin_amdgcn_s_memtime();                                        \
    if ((lane) == 0 && g_stamps) g_stamps[(size_t)block_env() * 48 + (slot)] = t_;               \
  } while (0)
// accumulate the cycles since `var` into slot (solver sub-phases), restart `var`
#define TSTART(var) unsigned long long var = __builtin_amdgcn_s_memtime()
#define TACC(slot, var, lane)                                                                    \
  do {                                                                                           \
    unsigned long long t_ = __builtin_amdgcn_s_memtime();                                        \
    if ((lane) == 0 && g_stamps) g_stamps[(size_t)block_env() * 48 + (slot)] += t_ - (var);      \
    (var) = t_;                                                                                  \
  } while (0)
#define TCOUNT(slot, n, lane)                                                                    \
  do {                                                                                           \
    if ((lane) == 0 && g_stamps) g_stamps[(size_t)block_env() * 48 + (slot)] += (n);             \
  } while (0)
#else
#define STAMP(slot, lane) do { } while (0)
#define TSTART(var) do { } while (0)
#define TACC(slot, var, lane) do { } while (0)
#define TCOUNT(slot, n, lane) do { } while (0)
#endif

typedef const CSTA ModelF* MP;

// LDS budget: 160 KB per CU / 8 waves (the VGPR limit at 2 waves per SIMD) = 20 KB per one-wave
// workgroup, so 2048 envs are resident on 256 CUs at once. Rows beyond CAP (contacts beyond CAPC)
// go to the env's global scratch slab.
#ifndef MJL_CAP
#define MJL_CAP 48
#endif
#ifndef MJL_CAPC
#define MJL_CAPC 16
#endif
#ifndef MJL_MINWAVES
#define MJL_MINWAVES 2
#endif
constexpr int kLdsBudget = 20480;
constexpr int CONW = 16;  // floats per contact record: pos[3], frame[9], then the pair's dof masks
                          // of both bodies, mu, and b1 | b2 << 8 | condim << 16 | k << 24 (int bits;
                          // k = which of a plane-capsule pair's two contacts)
constexpr float kMinVal = 1e-15f;
constexpr float kMinImp = 0.0001f;
constexpr float kMaxImp = 0.9999f;

// compile-time capacities of one kernel instantiation (model sizes must fit)
template <int NV_, int NB_, int NJ_, int NG_, int CAP_, int CAPC_> struct Dims {
  static constexpr int NV = NV_, NB = NB_, NJ = NJ_, NG = NG_, CAP = CAP_, CAPC = CAPC_;
  static constexpr int LD = (NV_ <= 28) ? 28 : 36;  // dense row stride, LD/4 odd -> conflict-free b128
};
using DHum = Dims<27, 17, 22, 20, MJL_CAP, MJL_CAPC>;  // both reference humanoids (nv 27, 17 bodies, 22 joints, 20 geoms)
using DGen = Dims<32, 32, 32, 32, 32, 16>;               // any model within the MJL_MAX* capacities
// the step VJP keeps its rows in the global slab, so its workspace drops the LDS row arrays (which
// share a union with the smooth-dynamics scratch): 6.4 KB less LDS, 5 instead of 4 waves per CU
using DHumV = Dims<27, 17, 22, 20, 4, 4>;

// ---------------------------------------------------------------------------------------------
// wave primitives
// ---------------------------------------------------------------------------------------------
INL float rdlane(float x, int k) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), k)); }
INL MP uniform_ptr(MP p) {
  unsigned long long v = (unsigned long long)p;
  unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return (MP)(((unsigned long long)hi << 32) | lo);
}
template <int CTRL, int ROWMASK> INL float dpp0(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROWMASK, 0xF, false));
}
template <int CTRL> INL float dppm(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
// sum over the 64 lanes, result in every lane (DPP within rows, row broadcasts, readlane 63)
INL float wsum(float v) {
  v += dppm<0xB1>(v);        // quad_perm 1,0,3,2
  v += dppm<0x4E>(v);        // quad_perm 2,3,0,1
  v += dppm<0x141>(v);       // row_half_mirror
  v += dppm<0x140>(v);       // row_mirror
  v += dpp0<0x142, 0xA>(v);  // row_bcast15
  v += dpp0<0x143, 0xC>(v);  // row_bcast31
  return rdlane(v, 63);
}
INL unsigned long long lanes_below(int lane) { return (1ull << lane) - 1ull; }
// The lane index through an opaque move: lane masks compared against it are computed where they
// are used. Against a plain lane index the compiler hoists a loop's 27 mask compares out of the
// Newton loop and spills them to VGPR lanes (two readlanes to restore each mask per use).
INL int opaque_int(int x) {
  int z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
  return x + z;
}

// a packed model record as whole b128 loads from the constant model block
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <class T> INL T ldrec(const CSTA T* p) {
  static_assert(sizeof(T) % 16 == 0, "records are 16-byte rows");
  union { u32x4 v[sizeof(T) / 16]; T t; } u;
  const CSTA u32x4* s = (const CSTA u32x4*)p;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 16); i++) u.v[i] = s[i];
  return u.t;
}

// ---------------------------------------------------------------------------------------------
// per-env LDS workspace
// ---------------------------------------------------------------------------------------------
// WS_HEAD / WS_TAIL: the workspace around its three dense-matrix arrays (M, H, invd). WSB<DM> is the
// same layout without them (the lean replay VJP reads those from the tape slot in global memory):
// every WSB field sits at its WS offset, shifted by the matrix block past the head.
#define WS_HEAD                                                                                      \
  static constexpr int NV = DM::NV, LD = DM::LD, NB = DM::NB, NJ = DM::NJ, NG = DM::NG;             \
  alignas(16) float qpos[MJL_MAXQ];                                                                \
  alignas(16) float qvel[LD];                                                                      \
  alignas(16) float qacc_ws[LD];                                                                   \
  float ctrl[MJL_MAXU];                                                                            \
  float xpos[NB][3], xquat[NB][4], xmat[NB][9], xipos[NB][3];                                      \
  float xanchor[NJ][3], xaxis[NJ][3];                                                              \
  float gpos[NG][3], gaxis[NG][3];                                                                 \
  float spos[MJL_MAXSITE][3], smat[MJL_MAXSITE][9];                                                \
  float scom[NB][3];                                                                               \
  float cdof[NV][6];                                                                               \
  float tenJ[MJL_MAXTENDON][LD], tenlen[MJL_MAXTENDON];
#define WS_TAIL                                                                                      \
  alignas(16) float frc_bias[LD];                                                                  \
  alignas(16) float frc_passive[LD];                                                               \
  alignas(16) float frc_act[LD];                                                                   \
  alignas(16) float frc_smooth[LD];                                                                \
  alignas(16) float qacc_smooth[LD];                                                               \
  alignas(16) float qacc[LD];                                                                      \
  alignas(16) float frc_con[LD];                                                                   \
  alignas(16) float grad[LD];                                                                      \
  alignas(16) float Mgrad[LD];                                                                     \
  alignas(16) float search[LD];                                                                    \
  alignas(16) float Ma[LD];                                                                        \
  alignas(16) float Mv[LD];                                                                        \
  alignas(16) float gradold[LD];                                                                   \
  alignas(16) float Mgradold[LD];                                                                  \
  float sens[MJL_MAXSENSOR];                                                                       \
  float sc[16];                                                                                    \
  int ncon, nefc, nlim, niter;                                                                     \
  static constexpr int CAP = DM::CAP, CAPC = DM::CAPC;                                             \
  union {                                                                                          \
    /* smooth-dynamics scratch: dead once the constraint rows are built */                         \
    struct { float cinert[NB][10], crb[NB][10], cvel[NB][6], cacc[NB][6]; };                       \
    /* constraint rows that fit in LDS */                                                          \
    struct {                                                                                       \
      alignas(16) float J[CAP * LD];                                                               \
      float D[CAP], aref[CAP], jar[CAP], force[CAP], Jv[CAP], epos[CAP], einvw[CAP];               \
      int emeta[CAP];                                                                              \
      float con[CAPC * CONW];                                                                      \
      int con_pair[CAPC], con_efc[CAPC];                                                           \
    };                                                                                             \
  };
template <class DM> struct WS {
  WS_HEAD
  alignas(16) float M[NV * LD];
  alignas(16) float H[NV * LD];  // factor of M, Newton Hessian + factor, or implicit-integration factor
  alignas(16) float invd[LD];    // 1 / diag of the factor in H
  WS_TAIL
};
template <class DM> struct WSB {  // WS without M, H, invd
  WS_HEAD
  WS_TAIL
};
static_assert(sizeof(WS<DHum>) <= kLdsBudget, "humanoid workspace exceeds the 8-waves-per-CU LDS budget");

// scalar slots in WS::sc
enum { SC_FLIP = 0, SC_HEIGHT, SC_ROLL, SC_PITCH, SC_YAW, SC_TF0, SC_TF1, SC_REW, SC_TERM, SC_TRUNC, SC_DONE,
       SC_NAN, SC_TIME, SC_NACT };

// constraint-row storage: the LDS arrays of WS, or the env's slab of global scratch
template <bool G> struct RowAS;
template <> struct RowAS<false> { typedef LDSA float F; typedef LDSA int I; };
template <> struct RowAS<true> { typedef GLBA float F; typedef GLBA int I; };
template <bool G> struct Rows {
  typedef typename RowAS<G>::F F;
  typedef typename RowAS<G>::I I;
  F *J, *D, *aref, *jar, *force, *Jv, *epos, *einvw, *con;
  I *emeta, *con_pair, *con_efc;
  int cap, capc;
};
template <class D> INL Rows<false> lds_rows(LDSA WS<D>* W) {
  Rows<false> R;
  R.J = W->J; R.D = W->D; R.aref = W->aref; R.jar = W->jar; R.force = W->force; R.Jv = W->Jv;
  R.epos = W->epos; R.einvw = W->einvw; R.emeta = W->emeta; R.con = W->con; R.con_pair = W->con_pair;
  R.con_efc = W->con_efc; R.cap = D::CAP; R.capc = D::CAPC;
  return R;
}
template <class D> INL Rows<true> global_rows(float* base_generic, int nefc_max, int ncon_max) {
  constexpr int LD = D::LD;
  GLBA float* p = (GLBA float*)base_generic;
  Rows<true> R;
  R.J = p; p += nefc_max * LD;
  R.D = p; p += nefc_max;
  R.aref = p; p += nefc_max;
  R.jar = p; p += nefc_max;
  R.force = p; p += nefc_max;
  R.Jv = p; p += nefc_max;
  R.epos = p; p += nefc_max;
  R.einvw = p; p += nefc_max;
  R.emeta = (GLBA int*)p; p += nefc_max;
  R.con = p; p += ncon_max * CONW;
  R.con_pair = (GLBA int*)p; p += ncon_max;
  R.con_efc = (GLBA int*)p;
  R.cap = nefc_max; R.capc = ncon_max;
  return R;
}

// ---------------------------------------------------------------------------------------------
// small math (MuJoCo conventions: quat [w x y z], spatial vectors [ang; lin], row-major 3x3)
// pointer arguments are templates so LDS / constant / private pointers all inline cleanly
// ---------------------------------------------------------------------------------------------
template <class A, class B> INL void qmul(float* r, A a, B b) {
  float t0 = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  float t1 = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  float t2 = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  float t3 = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3;
}
template <class Q> INL void q2m(float* m, Q q) {
  float w = q[0], x = q[1], y = q[2], z = q[3];
  m[0] = 1 - 2 * (y * y + z * z); m[1] = 2 * (x * y - w * z); m[2] = 2 * (x * z + w * y);
  m[3] = 2 * (x * y + w * z); m[4] = 1 - 2 * (x * x + z * z); m[5] = 2 * (y * z - w * x);
  m[6] = 2 * (x * z - w * y); m[7] = 2 * (y * z + w * x); m[8] = 1 - 2 * (x * x + y * y);
}
INL void qnorm(float* q) {
  float n = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < kMinVal) { q[0] = 1; q[1] = q[2] = q[3] = 0; return; }
  float inv = 1.f / n;
  q[0] *= inv; q[1] *= inv; q[2] *= inv; q[3] *= inv;
}
template <class M, class V> INL void mv3(float* r, M m, V v) {
  float a = m[0] * v[0] + m[1] * v[1] + m[2] * v[2];
  float b = m[3] * v[0] + m[4] * v[1] + m[5] * v[2];
  float c = m[6] * v[0] + m[7] * v[1] + m[8] * v[2];
  r[0] = a; r[1] = b; r[2] = c;
}
template <class M, class V> INL void mtv3(float* r, M m, V v) {
  float a = m[0] * v[0] + m[3] * v[1] + m[6] * v[2];
  float b = m[1] * v[0] + m[4] * v[1] + m[7] * v[2];
  float c = m[2] * v[0] + m[5] * v[1] + m[8] * v[2];
  r[0] = a; r[1] = b; r[2] = c;
}
template <class A, class B> INL void cross3(float* r, A a, B b) {
  float x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
  r[0] = x; r[1] = y; r[2] = z;
}
template <class A, class B> INL float dot3(A a, B b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
INL float norm3(float* v) {  // math.normalize_with_norm
  float n = sqrtf(dot3(v, v));
  float inv = 1.f / (n + (n == 0.f ? 1e-6f : 0.f));
  v[0] *= inv; v[1] *= inv; v[2] *= inv;
  return n;
}
template <class V, class U> INL void cross_motion(float* r, V v, U u) {
  float a[3], b[3], c[3];
  cross3(a, v, u); cross3(b, v, u + 3); cross3(c, v + 3, u);
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = b[0] + c[0]; r[4] = b[1] + c[1]; r[5] = b[2] + c[2];
}
template <class V, class F> INL void cross_force(float* r, V v, F f) {
  float a[3], b[3], c[3];
  cross3(a, v, f); cross3(b, v + 3, f + 3); cross3(c, v, f + 3);
  r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2]; r[3] = c[0]; r[4] = c[1]; r[5] = c[2];
}
template <class I, class V> INL void inert_vec(float* r, I i, V v) {
  r[0] = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
  r[1] = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
  r[2] = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
  r[3] = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
  r[4] = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
  r[5] = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
}

// ---------------------------------------------------------------------------------------------
// dense SPD factor / solve, one matrix row per lane in VGPRs (v_readlane broadcasts)
// ---------------------------------------------------------------------------------------------
// Factor the n x n SPD matrix A (LDS, stride LD) in place: A <- L (lower, upper zeroed),
// invd_out[i] = 1 / L[i][i]. Rows / cols >= n act as the identity.
template <class D> INL void chol_factor(LDSA float* A, LDSA float* invd_out, int n, int lane) {
  constexpr int NV = D::NV, LD = D::LD;
  float a[NV];
#pragma unroll
  for (int j = 0; j < NV; j++) a[j] = (lane < n && j < n) ? A[lane * LD + j] : (lane == j ? 1.f : 0.f);
  float invd = 1.f;
#pragma unroll
  for (int k = 0; k < NV; k++) {
    const float piv = fmaxf(rdlane(a[k], k), 1e-30f);
    const float inv = __builtin_amdgcn_rsqf(piv), lkk = piv * inv;
    a[k] = (lane == k) ? lkk : a[k] * inv;
    invd = (lane == k) ? inv : invd;
#pragma unroll
    for (int j = k + 1; j < NV; j++) a[j] = fmaf(-a[k], rdlane(a[k], j), a[j]);
  }
  if (lane < NV) {
#pragma unroll
    for (int j = 0; j < NV; j++) A[lane * LD + j] = (lane < n) ? ((j <= lane) ? a[j] : 0.f) : (j == lane ? 1.f : 0.f);
    invd_out[lane] = invd;
  }
  SYNC();
}

// One panel of the right-looking factor on rows held in registers (lane l and l + 32: row l & 31):
// columns [P0, P1) factored on the VALU (a readlane broadcast + fma per element), then their
// rank-(P1 - P0) update of the columns >= P1 as (P1 - P0) / 2 v_mfma_f32_32x32x2_f32, whose A and
// B operands are the lane's own registers. The MFMA result C has row r of C in column r of the C
// layout, i.e. C[i][j] sits in lane i (half (j >> 2) & 1) register (j & 3) + 4 (j >> 3); one
// v_permlane32_swap of a register with itself hands each lane both halves' values.
template <int LD, int NV, int P0, int P1> INL void chol_panel(float (&a)[LD], int kh) {
  static_assert(P0 % 2 == 0 && P1 <= NV && NV <= 32, "panels start on a K = 2 boundary");
#pragma unroll
  for (int k = P0; k < P1; k++) {
    // the column's broadcasts read the unscaled a_jk (they do not wait for the pivot's rsq) and
    // each lane's multiplier is L_ik / L_kk instead. No pivot floor: like MJX's cho_factor (and the
    // oracle), a non-SPD pivot is not patched; its NaN reaches the env's non-finite guard. (A floor
    // on the rsq was one more dependent op per column: ~8 cycles x 27 on the factor's chain.)
    const float inv = __builtin_amdgcn_rsqf(rdlane(a[k], k));
    float s[P1];
#pragma unroll
    for (int j = k + 1; j < P1; j++) s[j] = rdlane(a[k], j);
    a[k] *= inv;  // lane k: sqrt of its pivot
    const float t = a[k] * inv;
#pragma unroll
    for (int j = k + 1; j < P1; j++) a[j] = fmaf(-t, s[j], a[j]);
  }
  if constexpr (P1 < NV) {
    static_assert(P1 % 2 == 0, "interior panel ends on a K = 2 boundary");
    f32x16 acc;
#pragma unroll
    for (int v = 0; v < 16; v++) acc[v] = 0.f;
#pragma unroll
    for (int t = P0 / 2; t < P1 / 2; t++) {
      const float op = kh ? a[2 * t + 1] : a[2 * t];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(op, op, acc, 0, 0, 0);
    }
    float lo[16], hi[16];
#pragma unroll
    for (int v = 0; v < 16; v++) {
      bool used = false;
#pragma unroll
      for (int j = P1; j < NV; j++) used |= ((j & 3) + 4 * (j >> 3)) == v;
      if (used) {
        auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[v]), __float_as_uint(acc[v]), false, false);
        lo[v] = __uint_as_float(r[0]);
        hi[v] = __uint_as_float(r[1]);
      }
    }
#pragma unroll
    for (int j = P1; j < NV; j++) {
      const int v = (j & 3) + 4 * (j >> 3);
      a[j] -= ((j >> 2) & 1) ? hi[v] : lo[v];
    }
  }
}

// Factor + solve in one pass, for the hot callers (M in forward / integrate, the Newton Hessian):
// L L^T = S (S: n x n SPD in LDS at src, stride LD), L written to dst (lower triangle; the upper
// triangle is unspecified, chol_solve reads only the lower) with invd_out[i] = 1 / L[i][i];
// returns (L L^T)^-1 rhs with row i's value in lanes i and i + 32.
//
// nv < 32 (chol_aug_factor_solve): rows of S in VGPRs, lane l and l + 32 both holding row l & 31,
// and the right-hand side riding along as one more row, R = NV. The factor's own column
// broadcasts then run the forward substitution: lane R ends with L[R][k] = y_k (L y = rhs). The
// back substitution runs on the unit upper factor diag(L)^-1 L^T: lane i pre-scales its column
// L[k][i] (k > i) by its own 1 / L[i][i], so each of the NV serial steps is one readlane and one
// fma, with no lane masks in the chain. The factor runs in 8-column panels (chol_panel).
// Padding contract (n < NV): S is the identity outside its n x n block (M is built that way, and
// the Newton / implicit matrices inherit it) and rhs is zero beyond n.
// ADD: S = src + C, C a symmetric matrix in a v_mfma_f32_32x32x2_f32 accumulator (C layout: register
// v of lane l holds C[(v&3) + 8(v>>2) + 4(l>>5)][l&31], zero outside nv x nv): by symmetry lane c's
// registers hold row c at the columns of its half, and v_permlane32_swap hands it the other half's.
template <class D, bool ADD> INL float chol_aug_factor_solve(const LDSA float* src, LDSA float* dst,
                                                             LDSA float* invd_out, int n, const LDSA float* rhs,
                                                             int lane, f32x16 C = {}) {
  constexpr int NV = D::NV, LD = D::LD, R = NV;
  static_assert(NV < 32 && LD % 4 == 0 && LD > NV, "augmented factor needs a spare row and 16-B rows");
  const int i = lane & 31, kh = lane >> 5;
  (void)n;
  float a[LD];
  TSTART(tch);
  if constexpr (ADD) {
#pragma unroll
    for (int v = 0; v < 16; v++) {
      auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(C[v]), __float_as_uint(C[v]), false, false);
      const int j0 = (v & 3) + 8 * (v >> 2);
      if (j0 < LD) a[j0] = __uint_as_float(r[0]);
      if (j0 + 4 < LD) a[j0 + 4] = __uint_as_float(r[1]);
    }
  }
  {  // row i of S (lanes i < NV), the right-hand side (lanes >= NV; kept by lane R)
    const LDSA f32x4* rp = (const LDSA f32x4*)((i < NV) ? src + i * LD : rhs);
#pragma unroll
    for (int q = 0; q < LD / 4; q++) {
      const f32x4 v = rp[q];
#pragma unroll
      for (int e = 0; e < 4; e++) a[4 * q + e] = ADD ? a[4 * q + e] + v[e] : v[e];
    }
  }
  TACC(32, tch, lane);

  // panels [0, 8), [8, 16), [16, NV): a last MFMA update for the final few columns cost more than
  // it saved (tools/chol_micro.hip: boundaries 8/16 beat 8/16/24 by 5 %, 10/20 by 3 %)
  chol_panel<LD, NV, 0, (NV < 8 ? NV : 8)>(a, kh);
  if constexpr (NV > 8) chol_panel<LD, NV, 8, (NV < 16 ? NV : 16)>(a, kh);
  if constexpr (NV > 16) chol_panel<LD, NV, 16, NV>(a, kh);
  // rows of L to dst, y = L[R][0..NV) to invd_out (scratch until the reads below)
  TACC(33, tch, lane);
  if (lane <= R) {
    LDSA f32x4* wp = (LDSA f32x4*)((i == R) ? invd_out : dst + i * LD);
#pragma unroll
    for (int q = 0; q < LD / 4; q++) {
      f32x4 v;
      v[0] = a[4 * q]; v[1] = a[4 * q + 1]; v[2] = a[4 * q + 2]; v[3] = a[4 * q + 3];
      wp[q] = v;
    }
  }
  // No wait for the stores: one wave's LDS requests complete in order, so the column reads below
  // see them (the compiler keeps the reads after the stores to the same arrays). All reads are
  // unconditional (lanes >= NV read column 0 and mask it) and issue together, the back
  // substitution's first columns (k = NV - 1 ...) first.
  const int ic = (i < NV) ? i : 0;
  const float dg = dst[ic * LD + ic], yv = invd_out[ic];
  float w[NV];
#pragma unroll
  for (int k = NV - 1; k >= 0; k--) w[k] = dst[k * LD + ic];
  const float y = (i < NV) ? yv : 0.f;
  const float invd = (i < NV) ? __builtin_amdgcn_rcpf(dg) : 1.f;
  if (lane < NV) invd_out[lane] = invd;  // after the y read (same wave: LDS requests complete in order)
  TACC(34, tch, lane);
  const int io = opaque_int(i);
#pragma unroll
  for (int k = 0; k < NV; k++) w[k] = (io < k) ? w[k] * invd : 0.f;  // L[k][i] / L[i][i]
  float x = y * invd;
#pragma unroll
  for (int k = NV - 1; k >= 0; k--) x = fmaf(-w[k], rdlane(x, k), x);
  TACC(35, tch, lane);
  return x;
}

// nv = 32 (chol_rows_factor_solve, the generic instantiation): explicit forward substitution.
// Lanes l and l + 32 both hold row l & 31, so the trailing update of the two-block right-looking
// factorisation, S22 -= L21 L21^T over the first 16 columns, is 8 fp32 MFMAs whose A and B
// operands are the lane's own registers. The MFMA result C has row r of C in column r of the
// C layout, i.e. C[i][j] sits in lane i (half (j >> 2) & 1) register (j & 3) + 4 (j >> 3);
// v_permlane32_swap of a register with itself hands each lane both halves' values.
template <class D> INL float chol_rows_factor_solve(const LDSA float* src, LDSA float* dst, LDSA float* invd_out,
                                                    int n, const LDSA float* rhs, int lane) {
  constexpr int NV = D::NV, LD = D::LD;
  constexpr int B1 = NV > 16 ? 16 : NV;
  const int i = lane & 31, kh = lane >> 5;
  float a[NV];
#pragma unroll
  for (int j = 0; j < NV; j++) a[j] = (i < n && j < n) ? src[i * LD + j] : (i == j ? 1.f : 0.f);
  float x = (i < n) ? rhs[i] : 0.f;
  float invd = 1.f;
#pragma unroll
  for (int k = 0; k < B1; k++) {
    const float piv = fmaxf(rdlane(a[k], k), 1e-30f);
    const float inv = __builtin_amdgcn_rsqf(piv), lkk = piv * inv;
    a[k] = (i == k) ? lkk : a[k] * inv;
    invd = (i == k) ? inv : invd;
#pragma unroll
    for (int j = k + 1; j < B1; j++) a[j] = fmaf(-a[k], rdlane(a[k], j), a[j]);
  }
  if constexpr (NV > B1) {
    f32x16 acc;
#pragma unroll
    for (int v = 0; v < 16; v++) acc[v] = 0.f;
#pragma unroll
    for (int t = 0; t < B1 / 2; t++) {
      const float op = kh ? a[2 * t + 1] : a[2 * t];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(op, op, acc, 0, 0, 0);
    }
    float lo[16], hi[16];  // lo[v]: register v of the kh = 0 half, hi[v]: of the kh = 1 half
#pragma unroll
    for (int v = B1 / 2; v < 16; v++) {
      auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[v]), __float_as_uint(acc[v]), false, false);
      lo[v] = __uint_as_float(r[0]);
      hi[v] = __uint_as_float(r[1]);
    }
#pragma unroll
    for (int j = B1; j < NV; j++) {
      const int v = (j & 3) + 4 * (j >> 3);
      a[j] -= ((j >> 2) & 1) ? hi[v] : lo[v];
    }
#pragma unroll
    for (int k = B1; k < NV; k++) {
      const float piv = fmaxf(rdlane(a[k], k), 1e-30f);
      const float inv = __builtin_amdgcn_rsqf(piv), lkk = piv * inv;
      a[k] = (i == k) ? lkk : a[k] * inv;
      invd = (i == k) ? inv : invd;
#pragma unroll
      for (int j = k + 1; j < NV; j++) a[j] = fmaf(-a[k], rdlane(a[k], j), a[j]);
    }
  }
  if (lane < NV) {
#pragma unroll
    for (int j = 0; j < NV; j++) dst[i * LD + j] = (i < n) ? ((j <= i) ? a[j] : 0.f) : (j == i ? 1.f : 0.f);
    invd_out[i] = invd;
  }
  // forward substitution L y = rhs, from the rows in registers
#pragma unroll
  for (int k = 0; k < NV; k++) {
    const float yk = rdlane(x * invd, k);
    x = (i == k) ? yk : ((i > k) ? fmaf(-a[k], yk, x) : x);
  }
  SYNC();
  // back substitution L^T z = y: column i of L from the rows just written
  float lc[NV];
#pragma unroll
  for (int k = 0; k < NV; k++) lc[k] = (i < k) ? dst[k * LD + i] : 0.f;
#pragma unroll
  for (int k = NV - 1; k >= 0; k--) {
    const float zk = rdlane(x * invd, k);
    x = (i == k) ? zk : ((i < k) ? fmaf(-lc[k], zk, x) : x);
  }
  return x;
}

template <class D> INL float chol_factor_solve(const LDSA float* src, LDSA float* dst, LDSA float* invd_out,
                                               int n, const LDSA float* rhs, int lane) {
#ifndef MJL_CHOL_ROWS
  if constexpr (D::NV < 32) return chol_aug_factor_solve<D, false>(src, dst, invd_out, n, rhs, lane);
#endif
  return chol_rows_factor_solve<D>(src, dst, invd_out, n, rhs, lane);
}

// x distributed (lane i holds b_i, zero for i >= n) -> (L L^T)^-1 b, L from chol_factor
// unit-triangular forms, each lane scaling its own row / column by its own 1 / L[i][i]:
// L y = b  <=>  (diag(L)^-1 L) y = diag(L)^-1 b;  L^T z = y  <=>  (L diag(L)^-1)^T z = diag(L)^-1 y,
// so every serial step is one readlane and one fma. chol_load issues the lane's row and column of L
// (clamped addresses, loads unconditional; masks against an opaque lane index, see opaque_int) --
// callers with L in global memory issue it early, ahead of other work -- and chol_apply runs the two
// substitutions.
template <int NV> struct CholOps {
  float wr[NV], wc[NV], invd;
};
template <class D, class LP = const LDSA float*, class IP = const LDSA float*>
INL CholOps<D::NV> chol_load(LP L, IP invd_in, int lane) {
  constexpr int NV = D::NV, LD = D::LD;
  const int li = lane < NV ? lane : 0, lo = opaque_int(lane);
  CholOps<NV> c;
  c.invd = (lane < NV) ? invd_in[li] : 1.f;
#pragma unroll
  for (int k = 0; k < NV; k++) {
    const float r = L[li * LD + k], cl = L[k * LD + li];
    c.wr[k] = (lo < NV && lo > k) ? r * c.invd : 0.f;  // L[i][k] / L[i][i]
    c.wc[k] = (lo < k) ? cl * c.invd : 0.f;             // L[k][i] / L[i][i]
  }
  return c;
}
template <int NV> INL float chol_apply(const CholOps<NV>& c, float x) {
  x *= c.invd;
#pragma unroll
  for (int k = 0; k < NV; k++) x = fmaf(-c.wr[k], rdlane(x, k), x);
  x *= c.invd;
#pragma unroll
  for (int k = NV - 1; k >= 0; k--) x = fmaf(-c.wc[k], rdlane(x, k), x);
  return x;
}
template <class D, class LP = const LDSA float*, class IP = const LDSA float*>
INL float chol_solve(LP L, IP invd_in, float x, int lane) {  // L, invd in LDS, or in global memory (lean replay)
  return chol_apply(chol_load<D>(L, invd_in, lane), x);
}

// ---------------------------------------------------------------------------------------------
// position stage: kinematics, tendons, geom/site frames, subtree com   [smooth.kinematics]
// ---------------------------------------------------------------------------------------------
// The smooth phases' per-lane model records, issued together before the first of them waits (the
// kernel issues them before its state loads, so both latencies overlap): this lane's body, joint,
// the body's first three hinges, its geom / site frame constants and its dof (lane & 31).
struct KinPre {
  BodyRec br;       // brec[lane < nbody ? lane : 0]: kinematics, com_pos_crb, velocity_stage
  JntRec jown;      // jrec[lane < njnt ? lane : 0]
  HingeRec bh[3];   // the body's first three hinges
  FrameRec fr;      // geom lane (< 32) or site lane (32 + s)
  DofRec dr;        // drec[(lane & 31) < nv ? lane & 31 : 0]: com_pos_crb (cdof, M column), velocity_stage
};
INL KinPre kin_prefetch(MP m_, int lane) {
  MP m = uniform_ptr(m_);
  KinPre k;
  const int b = lane < m->nbody ? lane : 0;
  k.br = ldrec(&m->brec[b]);
  k.jown = ldrec(&m->jrec[lane < m->njnt ? lane : 0]);
#pragma unroll
  for (int i = 0; i < 3; i++) k.bh[i] = ldrec(&m->bhinge[b][i]);
  k.fr = ldrec(&m->frec[lane]);
  k.dr = ldrec(&m->drec[(lane & 31) < m->nv ? (lane & 31) : 0]);
  return k;
}

template <class D> PHASE void kinematics(MP m_, LDSA WS<D>* W, int lane, const KinPre& kp) {
  MP m = uniform_ptr(m_);
  const int maxlevel = m->maxlevel, nbody = m->nbody, ngeom = m->ngeom, nsite = m->nsite, njnt = m->njnt;
  TSTART(tk);
  // model records of this lane (kin_prefetch): body `lane`, geom `lane`, site `lane - 32`, joint `lane`
  const bool isb = lane > 0 && lane < nbody;
  const BodyRec& br = kp.br;
  const bool isg = lane < ngeom, iss = lane >= 32 && lane - 32 < nsite, isj = lane < njnt;
  const int gb = isg ? kp.fr.body : 0, sb = iss ? kp.fr.body : 0;
  const float* gp = kp.fr.pos;
  const float* gz = kp.fr.mat;
  const float* sp = kp.fr.pos;
  const float* sm = kp.fr.mat;
  const JntRec& jown = kp.jown;
  const int jpar = jown.parent, jfree = isj ? jown.isfree : 1;
  TACC(16, tk, lane);
  if (lane == 0) {
    W->xpos[0][0] = W->xpos[0][1] = W->xpos[0][2] = 0.f;
    W->xquat[0][0] = 1.f; W->xquat[0][1] = W->xquat[0][2] = W->xquat[0][3] = 0.f;
    for (int i = 0; i < 9; i++) W->xmat[0][i] = (i % 4 == 0) ? 1.f : 0.f;
    W->xipos[0][0] = W->xipos[0][1] = W->xipos[0][2] = 0.f;
  }
  if (lane >= 32 && lane - 32 < m->ntendon) {  // fixed tendons  [smooth.tendon]
    int t = lane - 32;
    float len = 0.f;
    for (int k = 0; k < D::LD; k++) W->tenJ[t][k] = 0.f;
    for (int w = 0; w < m->tendon_num[t]; w++) {
      len += m->tendon_coef[t][w] * W->qpos[m->tendon_qadr[t][w]];
      W->tenJ[t][m->tendon_dof[t][w]] += m->tendon_coef[t][w];
    }
    W->tenlen[t] = len;
  }
  // hinge rotations, one joint per lane (all sincos at once): ql_j = [cos(t/2), axis sin(t/2)]
  float jq[4] = {1.f, 0.f, 0.f, 0.f};
  if (isj && !jfree) {
    float s, c;
    sincosf(0.5f * (W->qpos[jown.qadr] - jown.qpos0), &s, &c);
    jq[0] = c; jq[1] = jown.axis[0] * s; jq[2] = jown.axis[1] * s; jq[3] = jown.axis[2] * s;
  }
  // a body's first three joints: hinge records from kin_prefetch, rotations from the joint lanes
  constexpr int KJ = 3;
  float ql3[KJ][4];
#pragma unroll
  for (int k = 0; k < KJ; k++) {
    const int j = (isb && k < br.jntnum) ? br.jntadr + k : 0;
#pragma unroll
    for (int e = 0; e < 4; e++) ql3[k][e] = __shfl(jq[e], j);
  }
  // body transform relative to its parent (lane = body, all bodies at once); hinge anchors and
  // axes are left in the parent frame in xanchor / xaxis and moved to world after the tree pass
  float lp[3], lq[4];
  if (isb) {
    if (br.isfree) {  // free joint: qpos is the world pose
      const int qa = br.qadr;
      lp[0] = W->qpos[qa]; lp[1] = W->qpos[qa + 1]; lp[2] = W->qpos[qa + 2];
      lq[0] = W->qpos[qa + 3]; lq[1] = W->qpos[qa + 4]; lq[2] = W->qpos[qa + 5]; lq[3] = W->qpos[qa + 6];
      qnorm(lq);
    } else {
      lp[0] = br.pos[0]; lp[1] = br.pos[1]; lp[2] = br.pos[2];
      lq[0] = br.quat[0]; lq[1] = br.quat[1]; lq[2] = br.quat[2]; lq[3] = br.quat[3];
#pragma unroll
      for (int k = 0; k < KJ; k++) {
        if (k >= br.jntnum) break;
        const int j = br.jntadr + k;
        const HingeRec& jr = kp.bh[k];
        float mat[9], anc[3], ax[3];
        q2m(mat, lq);
        mv3(anc, mat, jr.pos);
        anc[0] += lp[0]; anc[1] += lp[1]; anc[2] += lp[2];
        mv3(ax, mat, jr.axis);
        W->xanchor[j][0] = anc[0]; W->xanchor[j][1] = anc[1]; W->xanchor[j][2] = anc[2];
        W->xaxis[j][0] = ax[0]; W->xaxis[j][1] = ax[1]; W->xaxis[j][2] = ax[2];
        qmul(lq, lq, ql3[k]);
        float off[3];
        q2m(mat, lq);
        mv3(off, mat, jr.pos);
        lp[0] = anc[0] - off[0]; lp[1] = anc[1] - off[1]; lp[2] = anc[2] - off[2];
      }
      for (int j = br.jntadr + KJ; j < br.jntadr + br.jntnum; j++) {  // bodies with more hinges
        const JntRec jr = ldrec(&m->jrec[j]);
        float mat[9], anc[3], ax[3];
        q2m(mat, lq);
        mv3(anc, mat, jr.pos);
        anc[0] += lp[0]; anc[1] += lp[1]; anc[2] += lp[2];
        mv3(ax, mat, jr.axis);
        W->xanchor[j][0] = anc[0]; W->xanchor[j][1] = anc[1]; W->xanchor[j][2] = anc[2];
        W->xaxis[j][0] = ax[0]; W->xaxis[j][1] = ax[1]; W->xaxis[j][2] = ax[2];
        float s, c;
        sincosf(0.5f * (W->qpos[jr.qadr] - jr.qpos0), &s, &c);
        const float ql[4] = {c, jr.axis[0] * s, jr.axis[1] * s, jr.axis[2] * s};
        qmul(lq, lq, ql);
        float off[3];
        q2m(mat, lq);
        mv3(off, mat, jr.pos);
        lp[0] = anc[0] - off[0]; lp[1] = anc[1] - off[1]; lp[2] = anc[2] - off[2];
      }
    }
  }
  // (no barrier: the level pass below works in registers; the anchors / axes written above are read
  // after the next barrier)
  TACC(17, tk, lane);
  // tree pass: compose with the parent's world frame, one level at a time  [smooth.kinematics].
  // A body's frame stays in its lane's registers; children read it with ds_bpermute (no LDS
  // round trip and no barrier per level), the parent's rotation matrix recomputed from its quat.
  float bm[4] = {0.f, 0.f, 0.f, 0.f};  // this body's mass moment and mass
  float wp[3] = {0.f, 0.f, 0.f}, wq[4] = {1.f, 0.f, 0.f, 0.f};  // lane 0: the world frame
  {
    const int par = isb ? br.parent : 0;
    for (int L = 1; L <= maxlevel; L++) {
      float pp[3], pq[4];
#pragma unroll
      for (int i = 0; i < 3; i++) pp[i] = __shfl(wp[i], par);
#pragma unroll
      for (int i = 0; i < 4; i++) pq[i] = __shfl(wq[i], par);
      if (isb && br.level == L) {
        if (br.isfree) {
          wp[0] = lp[0]; wp[1] = lp[1]; wp[2] = lp[2];
          wq[0] = lq[0]; wq[1] = lq[1]; wq[2] = lq[2]; wq[3] = lq[3];
        } else {
          float pm[9];
          q2m(pm, pq);
          mv3(wp, pm, lp);
          wp[0] += pp[0]; wp[1] += pp[1]; wp[2] += pp[2];
          qmul(wq, pq, lq);
          qnorm(wq);
        }
      }
    }
  }
  if (isb) {
    float mat[9], ip[3];
    q2m(mat, wq);
    const int b = lane;
    for (int i = 0; i < 3; i++) W->xpos[b][i] = wp[i];
    for (int i = 0; i < 4; i++) W->xquat[b][i] = wq[i];
    for (int i = 0; i < 9; i++) W->xmat[b][i] = mat[i];
    mv3(ip, mat, br.ipos);
    ip[0] += wp[0]; ip[1] += wp[1]; ip[2] += wp[2];
    W->xipos[b][0] = ip[0]; W->xipos[b][1] = ip[1]; W->xipos[b][2] = ip[2];
    bm[0] = br.mass * ip[0]; bm[1] = br.mass * ip[1]; bm[2] = br.mass * ip[2];
    bm[3] = br.mass;
  }
  SYNC();
  TACC(18, tk, lane);
  if (isj) {  // joint anchors / axes to world (lane = joint)
    float anc[3], ax[3];
    if (jfree) {  // free joint: anchor = body position, axis = body z
      const int b = jown.body;
      for (int i = 0; i < 3; i++) { anc[i] = W->xpos[b][i]; ax[i] = W->xmat[b][3 * i + 2]; }
    } else {
      const float la[3] = {W->xanchor[lane][0], W->xanchor[lane][1], W->xanchor[lane][2]};
      const float lx[3] = {W->xaxis[lane][0], W->xaxis[lane][1], W->xaxis[lane][2]};
      mv3(anc, W->xmat[jpar], la);
      anc[0] += W->xpos[jpar][0]; anc[1] += W->xpos[jpar][1]; anc[2] += W->xpos[jpar][2];
      mv3(ax, W->xmat[jpar], lx);
    }
    for (int i = 0; i < 3; i++) { W->xanchor[lane][i] = anc[i]; W->xaxis[lane][i] = ax[i]; }
  }
  if (isg) {  // geom frames (lanes 0..31): centre + z axis is all collision needs
    float p[3], z[3];
    mv3(p, W->xmat[gb], gp);
    mv3(z, W->xmat[gb], gz);
    W->gpos[lane][0] = W->xpos[gb][0] + p[0]; W->gpos[lane][1] = W->xpos[gb][1] + p[1];
    W->gpos[lane][2] = W->xpos[gb][2] + p[2];
    W->gaxis[lane][0] = z[0]; W->gaxis[lane][1] = z[1]; W->gaxis[lane][2] = z[2];
  }
  if (iss) {  // site frames (lanes 32..)
    const int s = lane - 32;
    float p[3];
    mv3(p, W->xmat[sb], sp);
    W->spos[s][0] = W->xpos[sb][0] + p[0]; W->spos[s][1] = W->xpos[sb][1] + p[1]; W->spos[s][2] = W->xpos[sb][2] + p[2];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++)
        W->smat[s][3 * i + j] = W->xmat[sb][3 * i] * sm[j] + W->xmat[sb][3 * i + 1] * sm[3 + j] + W->xmat[sb][3 * i + 2] * sm[6 + j];
  }
  TACC(19, tk, lane);
  // subtree com of the kinematic roots, the only subtree com the dynamics reads (cinert, cdof and
  // contact Jacobians are taken about scom[rootid]); a root's subtree is lanes [r, subtree_end)
  for (int q = 0; q < m->nroot; q++) {
    const int r = m->root[q], e = m->body_subtree_end[r];
    const bool in = lane >= r && lane < e;
    const float s0 = wsum(in ? bm[0] : 0.f), s1 = wsum(in ? bm[1] : 0.f), s2 = wsum(in ? bm[2] : 0.f);
    const float ms = wsum(in ? bm[3] : 0.f);
    if (lane == 0) {
      if (ms < kMinVal) { W->scom[r][0] = W->xipos[r][0]; W->scom[r][1] = W->xipos[r][1]; W->scom[r][2] = W->xipos[r][2]; }
      else { const float inv = 1.f / ms; W->scom[r][0] = s0 * inv; W->scom[r][1] = s1 * inv; W->scom[r][2] = s2 * inv; }
    }
  }
  SYNC();
}

// Subtree sums over the DFS-contiguous body ranges, out[b][j] = sum_{c in [b, end_b)} in[c][j] for
// bodies 1..16 (nbody <= 17), as four v_mfma_f32_16x16x4_f32: A = the 0/1 subtree indicator
// (output body x contracted body), B = the per-body rows. Products with 0/1 and an f32
// accumulate chain in ascending body order: the same sums, bit for bit, as the serial loop.
// `end_lane`: this lane's body's subtree_end (lanes 1..16).
template <int NC, class Src, class Dst> INL void subtree_sums16(Src in, Dst out, int nbody, int end_lane, int lane) {
  const int bi = (lane & 15) + 1, k = lane >> 4, j = lane & 15;
  const int endb = __shfl(end_lane, bi);
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  f32x4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 4; t++) {
    const int c = 1 + k + 4 * t;
    const float a = (c >= bi && c < endb) ? 1.f : 0.f;
    const float bv = (c < nbody && j < NC) ? in[c][j] : 0.f;
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv, acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int b = 1 + 4 * k + r;
    if (b < nbody && j < NC) out[b][j] = acc[r];
  }
}

// cinert (lane = body) and cdof (lane 32 + dof); crb (lane = body); M columns (lane = dof)
template <class D> PHASE void com_pos_crb(MP m_, LDSA WS<D>* W, int lane, const KinPre& kp) {
  MP m = uniform_ptr(m_);
  constexpr int LD = D::LD;
  const int nbody = m->nbody, nv = m->nv;
  const bool isb = lane < nbody, iscd = lane >= 32 && lane - 32 < nv;
  const BodyRec& br = kp.br;
  const DofRec &dcd = kp.dr, &dcol = kp.dr;  // lanes 32 + d (cdof of dof d) and lane & 31 (M column)
  TSTART(tc);
  const float* t = br.inertia;
  if (isb) {
    const int b = lane;
    LDSA float* ci = W->cinert[b];
    const float mass = br.mass;
    if (b == 0 || mass == 0.f) {
      for (int i = 0; i < 10; i++) ci[i] = 0.f;
    } else {
      float X[9];
      for (int i = 0; i < 9; i++) X[i] = W->xmat[b][i];
      float Ib[9] = {t[0], t[3], t[4], t[3], t[1], t[5], t[4], t[5], t[2]};
      float T[9], Iw[9];
      for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) T[3 * i + j] = X[3 * i] * Ib[j] + X[3 * i + 1] * Ib[3 + j] + X[3 * i + 2] * Ib[6 + j];
      for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) Iw[3 * i + j] = T[3 * i] * X[3 * j] + T[3 * i + 1] * X[3 * j + 1] + T[3 * i + 2] * X[3 * j + 2];
      const int root = br.rootid;
      float c[3] = {W->xipos[b][0] - W->scom[root][0], W->xipos[b][1] - W->scom[root][1], W->xipos[b][2] - W->scom[root][2]};
      float cc = dot3(c, c);
      ci[0] = Iw[0] + mass * (cc - c[0] * c[0]);
      ci[1] = Iw[4] + mass * (cc - c[1] * c[1]);
      ci[2] = Iw[8] + mass * (cc - c[2] * c[2]);
      ci[3] = Iw[1] - mass * c[0] * c[1];
      ci[4] = Iw[2] - mass * c[0] * c[2];
      ci[5] = Iw[5] - mass * c[1] * c[2];
      ci[6] = mass * c[0]; ci[7] = mass * c[1]; ci[8] = mass * c[2]; ci[9] = mass;
    }
  }
  if (iscd) {
    const int d = lane - 32, j = dcd.jntid, b = dcd.bodyid, root = dcd.rootid, k = dcd.kfree;
    LDSA float* cd = W->cdof[d];
    float off[3] = {W->scom[root][0] - W->xanchor[j][0], W->scom[root][1] - W->xanchor[j][1],
                    W->scom[root][2] - W->xanchor[j][2]};
    if (k >= 0 && k < 3) {
      for (int i = 0; i < 6; i++) cd[i] = 0.f;
      cd[3 + k] = 1.f;
    } else {
      float ax[3];
      if (k >= 3) {
        ax[0] = W->xmat[b][k - 3]; ax[1] = W->xmat[b][3 + k - 3]; ax[2] = W->xmat[b][6 + k - 3];
      } else {
        ax[0] = W->xaxis[j][0]; ax[1] = W->xaxis[j][1]; ax[2] = W->xaxis[j][2];
      }
      float l[3];
      cross3(l, ax, off);
      cd[0] = ax[0]; cd[1] = ax[1]; cd[2] = ax[2]; cd[3] = l[0]; cd[4] = l[1]; cd[5] = l[2];
    }
  }
  SYNC();
  TACC(23, tc, lane);
  if (nbody <= 17) {  // bodies 1..16 on the matrix core (crb[0] is never read)
    subtree_sums16<10>(W->cinert, W->crb, nbody, br.subtree_end, lane);
  } else if (isb) {
    const int b = lane;
    float s[10];
    for (int i = 0; i < 10; i++) s[i] = 0.f;
    for (int c = b; c < br.subtree_end; c++)
      for (int i = 0; i < 10; i++) s[i] += W->cinert[c][i];
    for (int i = 0; i < 10; i++) W->crb[b][i] = s[i];
  }
  for (int i = lane; i < D::NV * LD; i += 64) W->M[i] = 0.f;
  if (lane >= nv && lane < D::NV) W->M[lane * LD + lane] = 1.f;  // padded rows / cols: the identity
  SYNC();
  TACC(24, tc, lane);
  {  // M[i][j] = cdof_j . (crb_body(i) cdof_i) for j in the ancestor chain of i  [smooth.crb / make_m]:
     // every product cdof_r . f_c at once as three v_mfma_f32_32x32x2_f32 (K = 6), lane (c, half)
     // supplying cdof_c[k] and f_c[k]; the lane holding column c keeps the rows in c's chain
    const int i = lane & 31, h = lane >> 5;
    const bool isdof = i < nv;
    float f[6], c6[6], cr[10];
    for (int k = 0; k < 6; k++) c6[k] = isdof ? W->cdof[i][k] : 0.f;
    for (int k = 0; k < 10; k++) cr[k] = isdof ? W->crb[dcol.bodyid][k] : 0.f;
    inert_vec(f, cr, c6);
    f32x16 acc;
#pragma unroll
    for (int v = 0; v < 16; v++) acc[v] = 0.f;
#pragma unroll
    for (int t = 0; t < 3; t++)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(h ? c6[2 * t + 1] : c6[2 * t], h ? f[2 * t + 1] : f[2 * t], acc, 0, 0, 0);
    const uint32_t anc = isdof ? dcol.ancmask : 0u;
#pragma unroll
    for (int v = 0; v < 16; v++) {
      const int row = (v & 3) + 8 * (v >> 2) + 4 * h;
      if ((anc >> row) & 1u) {
        const float val = acc[v] + (row == i ? dcol.armature : 0.f);
        W->M[i * LD + row] = val;
        W->M[row * LD + i] = val;
      }
    }
  }
  SYNC();
}

// ---------------------------------------------------------------------------------------------
// velocity stage: com_vel + rne forward pass by levels, backward by subtree ranges; passive
// forces and actuation   [smooth.com_vel / smooth.rne / passive.passive / forward.fwd_actuation]
// ---------------------------------------------------------------------------------------------
template <class D> PHASE void velocity_stage(MP m_, LDSA WS<D>* W, int lane, const KinPre& kp) {
  MP m = uniform_ptr(m_);
  const int maxlevel = m->maxlevel, nbody = m->nbody, nv = m->nv, nu = m->nu;
  const bool isb = lane > 0 && lane < nbody, isd = lane < nv, isu = lane < nu;
  const BodyRec& br = kp.br;
  const DofRec& dr = kp.dr;
  int udof = 0, ulim = 0;
  TSTART(tv);
  float ugear = 0.f, ulo = 0.f, uhi = 0.f;
  if (isu) {
    udof = m->actuator_dof[lane]; ulim = m->actuator_ctrllimited[lane]; ugear = m->actuator_gear[lane];
    ulo = m->actuator_ctrlrange[lane][0]; uhi = m->actuator_ctrlrange[lane][1];
  }
  if (lane == 0) {
    for (int i = 0; i < 6; i++) W->cvel[0][i] = 0.f;
    W->cacc[0][0] = W->cacc[0][1] = W->cacc[0][2] = 0.f;
    W->cacc[0][3] = -m->gravity[0]; W->cacc[0][4] = -m->gravity[1]; W->cacc[0][5] = -m->gravity[2];
  }
  // this body's joint terms (lane = body): cvel_b = cvel_p + S, cacc_b = cacc_p + cvel_p x U + T
  // with S = sum cdof qd, U = the part of S that gets a cdof_dot term, T = the in-body cross terms
  float S[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, U[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float T[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (isb) {
    const int da = br.dofadr, dn = br.dofnum;
    if (br.isfree) {  // translation first; the rotational cdof_dot use cvel after translation
      for (int k = 0; k < 3; k++)
        for (int i = 0; i < 6; i++) S[i] += W->cdof[da + k][i] * W->qvel[da + k];
      for (int k = 3; k < 6; k++)
        for (int i = 0; i < 6; i++) U[i] += W->cdof[da + k][i] * W->qvel[da + k];
      cross_motion(T, S, U);
      for (int i = 0; i < 6; i++) S[i] += U[i];
    } else {
      for (int k = 0; k < dn; k++) {
        float v[6], x[6];
        const float qd = W->qvel[da + k];
        for (int i = 0; i < 6; i++) v[i] = W->cdof[da + k][i] * qd;
        cross_motion(x, S, v);
        for (int i = 0; i < 6; i++) { T[i] += x[i]; U[i] += v[i]; S[i] += v[i]; }
      }
    }
  }
  // (no barrier: the level pass works in registers, and the world rows written above are read only
  // after the next one)
  TACC(25, tv, lane);
  // cvel / cacc by levels in registers, the parent's read with ds_bpermute (lane 0: the world,
  // cvel 0 and cacc = -gravity)
  float wv[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float wa[6] = {0.f, 0.f, 0.f, -m->gravity[0], -m->gravity[1], -m->gravity[2]};
  {
    const int par = isb ? br.parent : 0;
    for (int L = 1; L <= maxlevel; L++) {
      float cv[6], ca[6];
#pragma unroll
      for (int i = 0; i < 6; i++) { cv[i] = __shfl(wv[i], par); ca[i] = __shfl(wa[i], par); }
      if (isb && br.level == L) {
        float x[6];
        cross_motion(x, cv, U);
        for (int i = 0; i < 6; i++) { wv[i] = cv[i] + S[i]; wa[i] = ca[i] + x[i] + T[i]; }
      }
    }
  }
  TACC(26, tv, lane);
  // body forces cfrc = I*a + v x* (I*v), written over cacc
  float f[6];
  if (isb) {
    float f1[6], iv[6], f2[6], ci[10];
    for (int i = 0; i < 10; i++) ci[i] = W->cinert[lane][i];
    inert_vec(f1, ci, wa);
    inert_vec(iv, ci, wv);
    cross_force(f2, wv, iv);
    for (int i = 0; i < 6; i++) f[i] = f1[i] + f2[i];
    for (int i = 0; i < 6; i++) W->cacc[lane][i] = f[i];
  }
  SYNC();
  if (nbody <= 17) {  // subtree sums of cfrc into cvel (cvel is no longer needed)
    subtree_sums16<6>(W->cacc, W->cvel, nbody, br.subtree_end, lane);
  } else if (isb) {
    float s[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int c = lane; c < br.subtree_end; c++)
      for (int i = 0; i < 6; i++) s[i] += W->cacc[c][i];
    for (int i = 0; i < 6; i++) W->cvel[lane][i] = s[i];
  }
  if (lane < D::LD) W->frc_act[lane] = 0.f;
  SYNC();
  TACC(27, tv, lane);
  if (isu) {  // motors with joint transmission
    float c = W->ctrl[lane];
    if (ulim) c = fminf(fmaxf(c, ulo), uhi);
    atomicAdd((float*)&W->frc_act[udof], ugear * c);
  }
  if (isd) {
    LDSA float* c = W->cdof[lane];
    LDSA float* fb = W->cvel[dr.bodyid];
    W->frc_bias[lane] = c[0] * fb[0] + c[1] * fb[1] + c[2] * fb[2] + c[3] * fb[3] + c[4] * fb[4] + c[5] * fb[5];
    float pf = -dr.damping * W->qvel[lane];
    if (dr.qadr_spring >= 0) pf -= dr.stiffness * (W->qpos[dr.qadr_spring] - dr.qpos_spring);
    W->frc_passive[lane] = pf;
  }
  SYNC();
  if (isd) W->frc_smooth[lane] = W->frc_passive[lane] - W->frc_bias[lane] + W->frc_act[lane];
  SYNC();
}

// row . v over LD entries as four interleaved partial sums (four 7-long FMA chains, not one 28-long)
template <int LD, class RowF, class VF> INL float rowdot(RowF* a, VF* v) {
  float s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < LD; k++) s[k & 3] = fmaf(a[k], v[k], s[k & 3]);
  return (s[0] + s[1]) + (s[2] + s[3]);
}

// ---------------------------------------------------------------------------------------------
// collision (MJX collision_primitive semantics)
// ---------------------------------------------------------------------------------------------
INL void make_frame(float* fr, const float* a_in) {  // math.make_frame
  float a[3] = {a_in[0], a_in[1], a_in[2]};
  norm3(a);
  float b[3] = {0.f, 0.f, 0.f};
  if (a[1] > -0.5f && a[1] < 0.5f) b[1] = 1.f; else b[2] = 1.f;
  float ab = dot3(a, b);
  b[0] -= a[0] * ab; b[1] -= a[1] * ab; b[2] -= a[2] * ab;
  norm3(b);
  float c[3];
  cross3(c, a, b);
  for (int i = 0; i < 3; i++) { fr[i] = a[i]; fr[3 + i] = b[i]; fr[6 + i] = c[i]; }
}
INL void seg_point(float* r, const float* a, const float* b, const float* pt) {  // math.closest_segment_point
  float ab[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
  float ap[3] = {pt[0] - a[0], pt[1] - a[1], pt[2] - a[2]};
  float t = dot3(ap, ab) / (dot3(ab, ab) + 1e-6f);
  t = fminf(fmaxf(t, 0.f), 1.f);
  r[0] = a[0] + t * ab[0]; r[1] = a[1] + t * ab[1]; r[2] = a[2] + t * ab[2];
}
INL float sph_sph(float* pos, float* n, const float* p1, float r1, const float* p2, float r2) {
  n[0] = p2[0] - p1[0]; n[1] = p2[1] - p1[1]; n[2] = p2[2] - p1[2];
  float dist = norm3(n) - (r1 + r2);
  float s = r1 + dist * 0.5f;
  pos[0] = p1[0] + n[0] * s; pos[1] = p1[1] + n[1] * s; pos[2] = p1[2] + n[2] * s;
  return dist;
}

// candidate contact k (0/1) of pair p; returns false if the pair has no k-th contact
template <class D> INL bool collide(const PairRec& pr, LDSA WS<D>* W, int k, float& dist, float* pos, float* fr) {
  const int kind = pr.kind;
  if (k == 1 && kind != MJL_COL_PLANE_CAPSULE) return false;
  const int g1 = pr.g1, g2 = pr.g2;
  float x1[3] = {W->gpos[g1][0], W->gpos[g1][1], W->gpos[g1][2]};
  float x2[3] = {W->gpos[g2][0], W->gpos[g2][1], W->gpos[g2][2]};
  float z1[3] = {W->gaxis[g1][0], W->gaxis[g1][1], W->gaxis[g1][2]};
  float z2[3] = {W->gaxis[g2][0], W->gaxis[g2][1], W->gaxis[g2][2]};
  const float r1 = pr.r1, r2 = pr.r2, h1 = pr.h1, h2 = pr.h2;
  if (kind == MJL_COL_PLANE_SPHERE) {
    float d[3] = {x2[0] - x1[0], x2[1] - x1[1], x2[2] - x1[2]};
    dist = dot3(d, z1) - r2;
    float s = r2 + 0.5f * dist;
    pos[0] = x2[0] - z1[0] * s; pos[1] = x2[1] - z1[1] * s; pos[2] = x2[2] - z1[2] * s;
    make_frame(fr, z1);
    return true;
  }
  if (kind == MJL_COL_PLANE_CAPSULE) {
    const float* n = z1;
    float nd = dot3(n, z2);
    float b[3] = {z2[0] - n[0] * nd, z2[1] - n[1] * nd, z2[2] - n[2] * nd};
    float bn = norm3(b);
    if (bn < 0.5f) {
      b[0] = 0.f; b[1] = 0.f; b[2] = 0.f;
      if (n[1] > -0.5f && n[1] < 0.5f) b[1] = 1.f; else b[2] = 1.f;
    }
    float c[3];
    cross3(c, n, b);
    float sg = (k == 0) ? 1.f : -1.f;
    float sp[3] = {x2[0] + sg * z2[0] * h2, x2[1] + sg * z2[1] * h2, x2[2] + sg * z2[2] * h2};
    float d[3] = {sp[0] - x1[0], sp[1] - x1[1], sp[2] - x1[2]};
    dist = dot3(d, n) - r2;
    float s = r2 + 0.5f * dist;
    pos[0] = sp[0] - n[0] * s; pos[1] = sp[1] - n[1] * s; pos[2] = sp[2] - n[2] * s;
    for (int i = 0; i < 3; i++) { fr[i] = n[i]; fr[3 + i] = b[i]; fr[6 + i] = c[i]; }
    return true;
  }
  float pa[3], pb[3];
  if (kind == MJL_COL_SPHERE_SPHERE) {
    for (int i = 0; i < 3; i++) { pa[i] = x1[i]; pb[i] = x2[i]; }
  } else if (kind == MJL_COL_SPHERE_CAPSULE) {
    float a[3] = {x2[0] - z2[0] * h2, x2[1] - z2[1] * h2, x2[2] - z2[2] * h2};
    float bb[3] = {x2[0] + z2[0] * h2, x2[1] + z2[1] * h2, x2[2] + z2[2] * h2};
    for (int i = 0; i < 3; i++) pa[i] = x1[i];
    seg_point(pb, a, bb, x1);
  } else {  // capsule-capsule (math.closest_segment_to_segment_points)
    float a0[3], a1[3], b0[3], b1[3];
    for (int i = 0; i < 3; i++) {
      a0[i] = x1[i] - z1[i] * h1; a1[i] = x1[i] + z1[i] * h1;
      b0[i] = x2[i] - z2[i] * h2; b1[i] = x2[i] + z2[i] * h2;
    }
    float da[3] = {a1[0] - a0[0], a1[1] - a0[1], a1[2] - a0[2]};
    float db[3] = {b1[0] - b0[0], b1[1] - b0[1], b1[2] - b0[2]};
    float la = norm3(da), lb = norm3(db);
    float ha = la * 0.5f, hb = lb * 0.5f;
    float am[3], bm[3], tr[3];
    for (int i = 0; i < 3; i++) { am[i] = a0[i] + da[i] * ha; bm[i] = b0[i] + db[i] * hb; tr[i] = am[i] - bm[i]; }
    float dadb = dot3(da, db), datr = dot3(da, tr), dbtr = dot3(db, tr);
    float den = 1.f - dadb * dadb;
    float ta0 = (-datr + dadb * dbtr) / (den + 1e-6f);
    float tb0 = dbtr + ta0 * dadb;
    float ta = fminf(fmaxf(ta0, -ha), ha), tb = fminf(fmaxf(tb0, -hb), hb);
    float na[3], nb[3];
    for (int i = 0; i < 3; i++) { pa[i] = am[i] + da[i] * ta; pb[i] = bm[i] + db[i] * tb; }
    seg_point(na, a0, a1, pb);
    seg_point(nb, b0, b1, pa);
    float d1 = 0.f, d2 = 0.f;
    for (int i = 0; i < 3; i++) { d1 += (pb[i] - na[i]) * (pb[i] - na[i]); d2 += (pa[i] - nb[i]) * (pa[i] - nb[i]); }
    if (d1 < d2) { pa[0] = na[0]; pa[1] = na[1]; pa[2] = na[2]; }
    else { pb[0] = nb[0]; pb[1] = nb[1]; pb[2] = nb[2]; }
  }
  float n[3];
  dist = sph_sph(pos, n, pa, r1, pb, r2);
  make_frame(fr, n);
  return true;
}

// ---------------------------------------------------------------------------------------------
// constraint rows: limits, contacts; then per-row D / aref   [constraint.make_constraint]
// ---------------------------------------------------------------------------------------------
template <class P> INL void kbi(float tstep, P solref, P solimp, float pos, float& k, float& b, float& imp) {
  float timeconst = fmaxf(solref[0], 2.f * tstep), dampratio = solref[1];
  float dmin = fminf(fmaxf(solimp[0], kMinImp), kMaxImp);
  float dmax = fminf(fmaxf(solimp[1], kMinImp), kMaxImp);
  float width = fmaxf(kMinVal, solimp[2]);
  float mid = fminf(fmaxf(solimp[3], kMinImp), kMaxImp);
  float power = fmaxf(1.f, solimp[4]);
  k = 1.f / (dmax * dmax * timeconst * timeconst * dampratio * dampratio);
  b = 2.f / (dmax * timeconst);
  if (solref[0] <= 0.f) k = -solref[0] / (dmax * dmax);
  if (solref[1] <= 0.f) b = -solref[1] / dmax;
  float x = fabsf(pos) / width;
  float y;
  if (power == 2.f) {  // the default power: exact squares instead of powf
    y = (x < mid) ? (1.f / mid) * x * x : 1.f - (1.f / (1.f - mid)) * (1.f - x) * (1.f - x);
  } else {
    y = (x < mid) ? (1.f / powf(mid, power - 1.f)) * powf(x, power)
                  : 1.f - (1.f / powf(1.f - mid, power - 1.f)) * powf(1.f - x, power);
  }
  imp = dmin + y * (dmax - dmin);
  imp = fminf(fmaxf(imp, dmin), dmax);
  if (x > 1.f) imp = dmax;
}

// Builds limit and contact rows into R (capacity R.cap / R.capc). Returns false, without writing
// past capacity, when they do not fit; W->ncon / nefc always hold the true counts.
template <class D, bool G> PHASE bool build_rows(MP m_, LDSA WS<D>* W, Rows<G> R, int lane) {
  MP m = uniform_ptr(m_);
  constexpr int LD = D::LD;
  typedef typename Rows<G>::F RF;
  const int nv = m->nv, cap = R.cap, capc = R.capc;
  int nl = 0;
  TSTART(tr);
  // every model record of the pass issues here, before the first wait: the first trip's pair
  // records (the next trip's load while a trip collides) and the limit records
  PairRec pr_next = ldrec(&m->prec[lane < m->npair ? lane : 0]);
  const LimRec jl = ldrec(&m->jlim[lane < m->njnt ? lane : 0]);
  const LimRec tl = ldrec(&m->tlim[lane < m->ntendon ? lane : 0]);
  const float tstep = m->timestep;
  // A limit row's impedance is known at creation (its pos and parameters are in the creating lane's
  // registers): D is written there, and k imp / b wait in aref / Jv for the row loop below, which
  // forms aref once J is built (the same expression as before, so the same rounding).
  auto row_imp = [&](int r, float pos, float invw, const float* sr, const float* si) {
    float k, b, imp;
    kbi(tstep, sr, si, pos, k, b, imp);
    R.D[r] = 1.f / fmaxf(invw * (1.f - imp) / imp, kMinVal);
    R.aref[r] = k * imp;
    R.Jv[r] = b;
  };
  {  // joint limits (lane = joint), then tendon limits (lane = tendon), ballot-compacted
    bool act = false;
    float dist = 0.f, sgn = 0.f;
    if (lane < m->njnt && jl.on) {
      float q = W->qpos[jl.qadr];
      float dmin = q - jl.lo, dmax = jl.hi - q;
      dist = fminf(dmin, dmax);
      sgn = dmin < dmax ? 1.f : -1.f;
      act = dist - jl.margin < 0.f;
    }
    unsigned long long bal = __ballot(act);
    int r = __popcll(bal & lanes_below(lane));
    if (act && r < cap) {
      RF* Jr = R.J + r * LD;
      for (int k = 0; k < LD; k++) Jr[k] = 0.f;
      Jr[jl.dofadr] = sgn;
      R.epos[r] = dist - jl.margin;
      R.einvw[r] = jl.invweight;
      R.emeta[r] = (0 << 16) | lane;
      row_imp(r, dist - jl.margin, jl.invweight, jl.solref, jl.solimp);
    }
    nl = __popcll(bal);
    act = false;
    if (lane < m->ntendon && tl.on) {
      float len = W->tenlen[lane];
      float dmin = len - tl.lo, dmax = tl.hi - len;
      dist = fminf(dmin, dmax);
      sgn = dmin < dmax ? 1.f : -1.f;
      act = dist - tl.margin < 0.f;
    }
    bal = __ballot(act);
    r = nl + __popcll(bal & lanes_below(lane));
    if (act && r < cap) {
      RF* Jr = R.J + r * LD;
      for (int k = 0; k < LD; k++) Jr[k] = (k < nv) ? sgn * W->tenJ[lane][k] : 0.f;
      R.epos[r] = dist - tl.margin;
      R.einvw[r] = tl.invweight;
      R.emeta[r] = (1 << 16) | lane;
      row_imp(r, dist - tl.margin, tl.invweight, tl.solref, tl.solimp);
    }
    nl += __popcll(bal);
  }
  // contacts, emitted in (trip, k, pair) order: trip = 64 consecutive candidate pairs, k = which of a
  // pair's contacts (only plane-capsule pairs have a second). One (pair, k) item per lane; active
  // items compacted by ballots, rows per contact 1 (condim 1) or 4 (condim 3, pyramidal).
  int nc = 0, nr = nl;
  const int npair = m->npair;
  TACC(20, tr, lane);
  auto emit = [&](const PairRec& pr, int p, int k, bool isp) {
    bool act = false;
    float dist = 0.f, pos[3], fr[9];
    if (isp && collide(pr, W, k, dist, pos, fr)) act = dist - pr.includemargin < 0.f;
    unsigned long long b1 = __ballot(act && pr.condim == 1), b4 = __ballot(act && pr.condim != 1);
    unsigned long long below = lanes_below(lane);
    int slot = __popcll((b1 | b4) & below);
    int rbefore = __popcll(b1 & below) + 4 * __popcll(b4 & below);
    int rows = pr.condim == 1 ? 1 : 4;
    int c = nc + slot, r0 = nr + rbefore;
    if (act && c < capc && r0 + rows <= cap) {
      RF* cr = R.con + c * CONW;
      cr[0] = pos[0]; cr[1] = pos[1]; cr[2] = pos[2];
      for (int i = 0; i < 9; i++) cr[3 + i] = fr[i];
      cr[12] = __uint_as_float(pr.mask1); cr[13] = __uint_as_float(pr.mask2); cr[14] = pr.mu;
      cr[15] = __int_as_float(pr.b1 | (pr.b2 << 8) | (pr.condim << 16) | (k << 24));
      R.con_pair[c] = p;
      R.con_efc[c] = r0;
      float ep = dist - pr.includemargin, iw = pr.invweight;
      for (int q = 0; q < rows; q++) {
        R.epos[r0 + q] = ep;
        R.einvw[r0 + q] = iw;
        R.emeta[r0 + q] = (2 << 16) | p;
      }
    }
    nc += __popcll(b1 | b4);
    nr += __popcll(b1) + 4 * __popcll(b4);
  };
  // Broadphase: a lower bound of every (pair, k)'s distance from the geom centres (exact for the
  // plane pairs; |x1 - x2| - r1 - r2 - h1 - h2 otherwise, the capsules' half lengths h). Items whose
  // bound clears the pair's margin by kSlack (far above fp32 rounding) cannot touch; the rest,
  // usually far fewer than 64, run the exact tests in ONE compacted pass, lane j = the j-th item in
  // emission order, so contacts, rows and every computed value are those of the full pass.
  constexpr float kSlack = 1e-4f;
  constexpr int kMaxTrip = (MJL_MAXPAIR + 63) / 64;
  const int ntrip = (npair + 63) / 64;
  unsigned long long cm[2 * kMaxTrip];  // candidate items per (trip, k), uniform
  int ncand = 0;
#pragma unroll
  for (int t = 0; t < kMaxTrip; t++) {
    cm[2 * t] = cm[2 * t + 1] = 0ull;
    if (t < ntrip) {
      const int p = 64 * t + lane;
      const PairRec pr = pr_next;
      if (t + 1 < ntrip) pr_next = ldrec(&m->prec[p + 64 < npair ? p + 64 : 0]);
      const LDSA float* x1 = W->gpos[pr.g1];
      const LDSA float* x2 = W->gpos[pr.g2];
      const LDSA float* z1 = W->gaxis[pr.g1];
      const LDSA float* z2 = W->gaxis[pr.g2];
      const float d[3] = {x2[0] - x1[0], x2[1] - x1[1], x2[2] - x1[2]};
      float lb0, lb1 = 1e30f;
      if (pr.kind == MJL_COL_PLANE_SPHERE || pr.kind == MJL_COL_PLANE_CAPSULE) {
        const float c = dot3(d, z1) - pr.r2, e = pr.h2 * dot3(z2, z1);
        lb0 = c + e;  // the exact plane distances of the (capsule end) points
        lb1 = pr.kind == MJL_COL_PLANE_CAPSULE ? c - e : 1e30f;
      } else {
        lb0 = sqrtf(dot3(d, d)) - pr.r1 - pr.r2 - pr.h1 - pr.h2;
      }
      const bool isp = p < npair;
      cm[2 * t] = __ballot(isp && lb0 - pr.includemargin < kSlack);
      cm[2 * t + 1] = __ballot(isp && lb1 - pr.includemargin < kSlack);
      ncand += __popcll(cm[2 * t]) + __popcll(cm[2 * t + 1]);
    }
  }
  if (ncand <= 64) {
    // lane j -> the j-th set bit of the concatenated masks (group g = 2 trip + k, then bit order)
    int g = 0, pre_g = 0, pre = 0;
#pragma unroll
    for (int q = 0; q < 2 * kMaxTrip; q++) {
      const int c = __popcll(cm[q]);
      if (q < 2 * ntrip && lane >= pre + c) { g = q + 1; pre_g = pre + c; }
      pre += c;
    }
    int r = lane - pre_g;
    unsigned long long mk = 0ull;
#pragma unroll
    for (int q = 0; q < 2 * kMaxTrip; q++) mk = (g == q) ? cm[q] : mk;
    // r-th set bit of mk (binary search on popcounts)
    unsigned w = (unsigned)mk;
    int pos = 0, cnt = __popc(w);
    if (r >= cnt) { r -= cnt; pos = 32; w = (unsigned)(mk >> 32); }
#pragma unroll
    for (int sh = 16; sh >= 1; sh >>= 1) {
      cnt = __popc(w & ((1u << sh) - 1u));
      if (r >= cnt) { r -= cnt; pos += sh; w >>= sh; }
    }
    const bool has = lane < ncand;
    const int p = has ? 64 * (g >> 1) + pos : 0, k = g & 1;
    const PairRec pr = ldrec(&m->prec[p]);
    emit(pr, p, k, has);
  } else {  // every item, trip by trip (records reloaded: the rare crowded state)
    for (int base = 0; base < npair; base += 64) {
      const int p = base + lane;
      const PairRec pr = ldrec(&m->prec[p < npair ? p : 0]);
      for (int k = 0; k < 2; k++) emit(pr, p, k, p < npair);
    }
  }
  if (lane == 0) { W->ncon = nc; W->nefc = nr; W->nlim = nl; }
  SYNC();
  TACC(21, tr, lane);
  if (nr > cap || nc > capc) return false;
  // contact Jacobian rows: lanes 0..31 -> contact c, lanes 32..63 -> contact c+1; lane%32 = dof
  const int d = lane & 31;
  const int droot = ldrec(&m->drec[d < nv ? d : 0]).rootid;
  for (int c0 = 0; c0 < nc; c0 += 2) {
    int c = c0 + (lane >> 5);
    if (c < nc && d < LD) {
      RF* cr = R.con + c * CONW;
      const uint32_t mask1 = __float_as_uint(cr[12]), mask2 = __float_as_uint(cr[13]);
      const int dim = (__float_as_int(cr[15]) >> 16) & 0xff;
      int r0 = R.con_efc[c];
      float vn = 0.f, vt1 = 0.f, vt2 = 0.f;
      if (d < nv) {
        float s = (float)((mask2 >> d) & 1u) - (float)((mask1 >> d) & 1u);
        if (s != 0.f) {
          float cd[6];
          for (int i = 0; i < 6; i++) cd[i] = W->cdof[d][i];
          float off[3] = {cr[0] - W->scom[droot][0], cr[1] - W->scom[droot][1], cr[2] - W->scom[droot][2]};
          float cx[3];
          cross3(cx, cd, off);
          float jp[3] = {s * (cd[3] + cx[0]), s * (cd[4] + cx[1]), s * (cd[5] + cx[2])};
          vn = cr[3] * jp[0] + cr[4] * jp[1] + cr[5] * jp[2];
          vt1 = cr[6] * jp[0] + cr[7] * jp[1] + cr[8] * jp[2];
          vt2 = cr[9] * jp[0] + cr[10] * jp[1] + cr[11] * jp[2];
        }
      }
      if (dim == 1) {
        R.J[r0 * LD + d] = vn;
      } else {
        const float mu = cr[14];
        R.J[(r0 + 0) * LD + d] = vn + mu * vt1;
        R.J[(r0 + 1) * LD + d] = vn - mu * vt1;
        R.J[(r0 + 2) * LD + d] = vn + mu * vt2;
        R.J[(r0 + 3) * LD + d] = vn - mu * vt2;
      }
    }
  }
  SYNC();
  TACC(22, tr, lane);
  // reference acceleration (lane = row): aref = -b J qvel - k imp pos; a limit row's b and k imp
  // from row_imp, a contact row's impedance here (lane = row: one pass for all contact rows)
  for (int r = lane; r < nr; r += 64) {
    const float pos = R.epos[r];
    float b, kimp;
    if (r >= nl) {
      const int id = R.emeta[r] & 0xffff;
      float k, imp;
      kbi(tstep, m->pair_solref[id], m->pair_solimp[id], pos, k, b, imp);
      R.D[r] = 1.f / fmaxf(R.einvw[r] * (1.f - imp) / imp, kMinVal);
      kimp = k * imp;
    } else {
      b = R.Jv[r];
      kimp = R.aref[r];
    }
    float vel = 0.f;
#pragma unroll
    for (int kk = 0; kk < LD; kk++) vel += R.J[r * LD + kk] * W->qvel[kk];
    R.aref[r] = -b * vel - kimp * pos;
  }
  SYNC();
  return true;
}

// ---------------------------------------------------------------------------------------------
// primal solver (Newton with exact line search; CG with Polak-Ribiere)   [solver.solve]
// ---------------------------------------------------------------------------------------------
template <class D> INL float mrow(LDSA WS<D>* W, LDSA float* v, int lane) {  // (M v)[lane]
  return rowdot<D::LD>(W->M + lane * D::LD, v);
}
template <class D, class RowF> INL float jrow(RowF* J, LDSA float* v, int r) {  // (J v)[r]
  return rowdot<D::LD>(J + r * D::LD, v);
}

// forces, cost, qfrc_constraint and gradient at the current qacc / Ma / jar; returns the cost and
// |grad|^2 (two wave sums issued together)
template <class D, bool G> INL float solver_update(MP m_, LDSA WS<D>* W, Rows<G> R, int lane, float& gsq) {
  MP m = uniform_ptr(m_);
  constexpr int LD = D::LD;
  const int nv = m->nv, nefc = W->nefc;
  // clamped indices throughout: each group of loads issues before its first use
  float c = 0.f;
  {
    const int ri = lane < nefc ? lane : 0;
    const float j = R.jar[ri], dr = R.D[ri];
    const bool act = lane < nefc && j < 0.f;
    if (lane < nefc) R.force[lane] = act ? -dr * j : 0.f;
    c = act ? 0.5f * dr * j * j : 0.f;
  }
  for (int r = lane + 64; r < nefc; r += 64) {
    float j = R.jar[r];
    float f = j < 0.f ? -R.D[r] * j : 0.f;
    R.force[r] = f;
    if (j < 0.f) c += 0.5f * R.D[r] * j * j;
  }
  const int mi = lane < nv ? lane : 0;
  const float ma = W->Ma[mi], fs = W->frc_smooth[mi], qa = W->qacc[mi], qsm = W->qacc_smooth[mi];
  SYNC();
  const int d = lane & 31, h = lane >> 5;  // J' f : lane%32 = dof, lane/32 = row parity
  float s = 0.f;
  if (d < nv) {
    int r = h;
    for (; r + 6 < nefc; r += 8)  // 4 rows per trip: the loads issue together
      s += R.J[r * LD + d] * R.force[r] + R.J[(r + 2) * LD + d] * R.force[r + 2] +
           R.J[(r + 4) * LD + d] * R.force[r + 4] + R.J[(r + 6) * LD + d] * R.force[r + 6];
    for (; r < nefc; r += 2) s += R.J[r * LD + d] * R.force[r];
  }
  s += __shfl_xor(s, 32);
  float g = 0.f, gr = 0.f;
  if (lane < nv) {
    W->frc_con[lane] = s;
    g = 0.5f * (ma - fs) * (qa - qsm);
    gr = ma - fs - s;
    W->grad[lane] = gr;
  }
  float cost = wsum(g + c);
  gsq = wsum(gr * gr);
  SYNC();
  return cost;
}

// Newton Hessian H = M + J' D_active J (factored by the caller), on the matrix cores:
// v_mfma_f32_32x32x2_f32 takes two constraint rows per instruction, lane l supplying
// A[i][k] = D_r J[r][i] (active rows only) and B[k][j] = J[r][j] with i = j = l & 31, r = r0 + (l >> 5);
// the 32x32 accumulator (nv <= 32) is H - M in the C layout row = (v&3) + 8(v>>2) + 4(l>>5), col = l&31.
template <class D, bool G> INL f32x16 solver_hessian_acc(MP m_, LDSA WS<D>* W, Rows<G> R, int lane) {
  MP m = uniform_ptr(m_);
  constexpr int LD = D::LD;
  const int nv = m->nv, nefc = W->nefc;
  const int col = lane & 31, kh = lane >> 5;
  f32x16 acc;
#pragma unroll
  for (int v = 0; v < 16; v++) acc[v] = 0.f;
#ifndef MJL_HESS_DENSE
  // only active rows (jar < 0) contribute: take them in order from each 64-row ballot, 8 rows per
  // trip (uniform row indices from s_ff1), loads of the trip first, then one MFMA per row pair
  for (int base = 0; base < nefc; base += 64) {
    unsigned long long am = __ballot(base + lane < nefc && R.jar[base + lane] < 0.f);
    while (am) {
      int rr[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        rr[u] = am ? base + (int)__builtin_ctzll(am) : -1;
        am &= am - 1;
      }
      float a[4], b[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int r = kh ? rr[2 * u + 1] : rr[2 * u];
        const bool ok = r >= 0 && col < nv;
        const int rs = r >= 0 ? r : 0;
        const float j = R.J[rs * LD + col];
        const float dr = R.D[rs];
        b[u] = ok ? j : 0.f;
        a[u] = ok ? dr * j : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; u++)
        if (rr[2 * u] >= 0) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u], b[u], acc, 0, 0, 0);
    }
  }
  return acc;
#endif
  for (int r0 = 0; r0 < nefc; r0 += 8) {
    float a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {  // loads of 4 row pairs first, then 4 MFMAs
      const int r = r0 + 2 * u + kh;
      a[u] = 0.f; b[u] = 0.f;
      if (r < nefc && col < nv) {
        const float j = R.J[r * LD + col];
        b[u] = j;
        a[u] = R.jar[r] < 0.f ? R.D[r] * j : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < 4; u++) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u], b[u], acc, 0, 0, 0);
  }
  return acc;
}
template <class D, bool G> INL void solver_hessian(MP m_, LDSA WS<D>* W, Rows<G> R, int lane) {
  constexpr int LD = D::LD;
  const int nv = uniform_ptr(m_)->nv;
  const int col = lane & 31, kh = lane >> 5;
  const f32x16 acc = solver_hessian_acc<D, G>(m_, W, R, lane);
#pragma unroll
  for (int v = 0; v < 16; v++) {
    const int row = (v & 3) + 8 * (v >> 2) + 4 * kh;
    if (row < nv && col < nv) W->H[row * LD + col] = W->M[row * LD + col] + acc[v];
  }
  SYNC();
}

// MJX's zoom line search along `search` (mujoco-mjx 3.3.6 solver.py _linesearch, restated in
// oracle/physics.hpp Solver::linesearch): bracket ends lo / hi around the root of f'(alpha); each
// iteration evaluates the Newton steps from both ends and the midpoint (one pass over the rows for
// all three points) and moves the ends by MJX's swap rules, until no end moves, an end's |f'| <
// gtol, or ls_iterations. Returns the lower-cost end if it improves on alpha = 0, else 0.
// Costs are relative to the Gauss term at alpha = 0 (common to every point, so comparisons hold).
// TP: tape hooks (NoTape in the primal kernels; the APG VJP's unrolled mode records every Newton
// point's parent active set and the accepted alpha's weights over them, adjoint.hip SolveTape).
template <class D, bool G, class TP> INL float solver_linesearch(MP m_, LDSA WS<D>* W, Rows<G> R, int lane, TP& tp) {
  MP m = uniform_ptr(m_);
  TSTART(tl);
  const int nv = m->nv, nefc = W->nefc;
  // M s, J s (the first 128 rows' J s, jar and D stay in registers across the iterations)
  // (clamped row indices: the M s and J s loads issue together, no branch between them)
  const int mi = lane < nv ? lane : 0, ri = lane < nefc ? lane : 0;
  const float mva = mrow<D>(W, W->search, mi), jva = jrow<D>(R.J, W->search, ri);
  const float sv = (lane < nv) ? W->search[mi] : 0.f;
  const float mvl = (lane < nv) ? mva : 0.f;
  const float c1p = sv * (W->Ma[mi] - W->frc_smooth[mi]), c2p = sv * mvl;
  if (lane < nv) W->Mv[lane] = mvl;
  float jv0 = 0.f, ja0 = 0.f, dd0 = 0.f, jv1 = 0.f, ja1 = 0.f, dd1 = 0.f;
  {
    const float ja = R.jar[ri], dd = R.D[ri];
    if (lane < nefc) { jv0 = jva; ja0 = ja; dd0 = dd; R.Jv[lane] = jv0; }
  }
  if (lane + 64 < nefc) {
    jv1 = jrow<D>(R.J, W->search, lane + 64); ja1 = R.jar[lane + 64]; dd1 = R.D[lane + 64]; R.Jv[lane + 64] = jv1;
  }
  for (int r = lane + 128; r < nefc; r += 64) R.Jv[r] = jrow<D>(R.J, W->search, r);
  // (Mv / Jv entries are read back only by the lanes that wrote them: no barrier in the primal)
  if constexpr (TP::on) SYNC();
  if constexpr (TP::on) tp.ls_begin(W, lane);
  TACC(28, tl, lane);
  // the step qacc += a s, Ma += a M s, jar += a J s from the registers the search already holds
  auto apply = [&](float alpha) -> float {
    if (alpha != 0.f) {
      if (lane < nv) { W->qacc[lane] += alpha * sv; W->Ma[lane] += alpha * mvl; }
      if (lane < nefc) R.jar[lane] = ja0 + alpha * jv0;
      if (lane + 64 < nefc) R.jar[lane + 64] = ja1 + alpha * jv1;
      for (int r = lane + 128; r < nefc; r += 64) R.jar[r] += alpha * R.Jv[r];
    }
    return alpha;
  };
  // lane partial sums of f'(al[k]), f''(al[k]) for K points (COST: of the relative cost), one
  // pass over the rows; `fin` turns them into the values (wave sums)
  auto partial = [&](auto Kc, auto COSTc, const float* al, float* dp, float* hp) {
    constexpr int K = decltype(Kc)::value;
    constexpr bool COST = decltype(COSTc)::value;
#pragma unroll
    for (int k = 0; k < K; k++) { dp[k] = 0.f; hp[k] = 0.f; }
    auto row = [&](float ja, float jv, float dd) {
#pragma unroll
      for (int k = 0; k < K; k++) {
        float j = ja + al[k] * jv;
        if (j < 0.f) {
          if (COST) { dp[k] += dd * j * j; } else { float dj = dd * jv; dp[k] += dj * j; hp[k] += dj * jv; }
        }
      }
    };
    row(ja0, jv0, dd0);
    row(ja1, jv1, dd1);
    for (int r = lane + 128; r < nefc; r += 64) row(R.jar[r], R.Jv[r], R.D[r]);
  };
  float c1 = 0.f, c2 = 0.f;
  auto fin = [&](auto Kc, auto COSTc, const float* al, const float* dp, const float* hp, float* o0, float* o1) {
    constexpr int K = decltype(Kc)::value;
    constexpr bool COST = decltype(COSTc)::value;
#pragma unroll
    for (int k = 0; k < K; k++) {
      if (COST) {
        o0[k] = al[k] * c1 + 0.5f * al[k] * al[k] * c2 + 0.5f * wsum(dp[k]);
      } else {
        o0[k] = c1 + al[k] * c2 + wsum(dp[k]);
        float h = c2 + wsum(hp[k]);
        o1[k] = h + (h == 0.f ? kMinVal : 0.f);
      }
    }
  };
  auto eval = [&](auto Kc, auto COSTc, const float* al, float* o0, float* o1) {
    constexpr int K = decltype(Kc)::value;
    float dp[K], hp[K];
    partial(Kc, COSTc, al, dp, hp);
    fin(Kc, COSTc, al, dp, hp, o0, o1);
  };
  using I1 = std::integral_constant<int, 1>;
  using I3 = std::integral_constant<int, 3>;
  using TF = std::false_type;
  using TT = std::true_type;
  // |s|, the Gauss terms c1 = s'(Ma - f), c2 = s'Ms and p0 = f'(0), f''(0): one batch of wave sums
  float a0[1] = {0.f}, p0d0[1], p0d1[1], snorm;
  {
    float dp[1], hp[1];
    partial(I1{}, TF{}, a0, dp, hp);
    snorm = sqrtf(wsum(sv * sv));
    c1 = wsum(c1p);
    c2 = wsum(c2p);
    fin(I1{}, TF{}, a0, dp, hp, p0d0, p0d1);
  }
  const float gtol = m->tolerance * m->ls_tolerance * snorm / m->scale;
  TACC(29, tl, lane);
  // the Newton point q from p0
  float a1[1] = {-p0d0[0] * __builtin_amdgcn_rcpf(p0d1[0])}, qd0[1], qd1[1];
  // tape: a point's alpha as weights over the recorded parent sets (lane j = set j); p0's alpha is 0
  float rec_q = 0.f, rec_lo = 0.f, rec_hi = 0.f;
  if constexpr (TP::on) rec_q = (lane == tp.add_set(R, nefc, 0.f, p0d1[0], a1[0], ja0, jv0, ja1, jv1, lane)) ? 1.f : 0.f;
  // exact segment: if no row changes activity between 0 and q, f' is linear there and q is its
  // root, the minimiser MJX's iterations then only jitter around in rounding noise
  {
    bool same = ((ja0 < 0.f) == (ja0 + a1[0] * jv0 < 0.f)) && ((ja1 < 0.f) == (ja1 + a1[0] * jv1 < 0.f));
    for (int r = lane + 128; r < nefc; r += 64) same &= (R.jar[r] < 0.f) == (R.jar[r] + a1[0] * R.Jv[r] < 0.f);
    if (__ballot(!same) == 0ull) {
      TCOUNT(15, 1, lane);
      if constexpr (TP::on) tp.ls_end(a1[0], rec_q, lane);
      return apply(a1[0]);
    }
  }
  eval(I1{}, TF{}, a1, qd0, qd1);
  TACC(30, tl, lane);
  // lo = whichever of p0, q has the smaller f'
  float loa, lod0, lod1, hia, hid0, hid1;
  if (qd0[0] < p0d0[0]) { loa = a1[0]; lod0 = qd0[0]; lod1 = qd1[0]; hia = 0.f; hid0 = p0d0[0]; hid1 = p0d1[0]; }
  else { loa = 0.f; lod0 = p0d0[0]; lod1 = p0d1[0]; hia = a1[0]; hid0 = qd0[0]; hid1 = qd1[0]; }
  if constexpr (TP::on) { if (qd0[0] < p0d0[0]) rec_lo = rec_q; else rec_hi = rec_q; }
  // MJX's gtol (tolerance * ls_tolerance * |search|) sits below the fp32 resolution of f', where
  // MJX's fp32 iterations only shuffle lo / hi within rounding noise until ls_iterations: an end
  // also counts as converged once |f'| is within kNoise of the magnitude of the terms summed into
  // it (|c1| + |a| f'' + |row part|), and the search stops once the bracket is a few ulps wide
  constexpr float kNoise = 2e-6f;
  auto tol = [&](float a, float d0, float d1) {
    return fmaxf(gtol, kNoise * (fabsf(c1) + fabsf(a) * d1 + fabsf(d0 - c1 - a * d1)));
  };
  float lot = tol(loa, lod0, lod1), hit = tol(hia, hid0, hid1);
  const int lsit = m->ls_iterations;
  for (int it = 0; it < lsit; it++) {
    if ((lod0 < 0.f && lod0 > -lot) || (hid0 > 0.f && hid0 < hit)) break;
    if (fabsf(hia - loa) <= 1e-6f * fmaxf(fabsf(loa), fabsf(hia))) break;
    float al[3] = {loa - lod0 * __builtin_amdgcn_rcpf(lod1), hia - hid0 * __builtin_amdgcn_rcpf(hid1), 0.5f * (loa + hia)};
    float rc[3] = {0.f, 0.f, 0.f};
    if constexpr (TP::on) {
      rc[0] = (lane == tp.add_set(R, nefc, loa, lod1, al[0], ja0, jv0, ja1, jv1, lane)) ? 1.f : 0.f;
      rc[1] = (lane == tp.add_set(R, nefc, hia, hid1, al[1], ja0, jv0, ja1, jv1, lane)) ? 1.f : 0.f;
      rc[2] = 0.5f * (rec_lo + rec_hi);
    }
    float d0[3], d1[3];
    eval(I3{}, TF{}, al, d0, d1);
    bool s1 = lod0 > 0.f || lod0 < d0[0];
    if (s1) { loa = al[0]; lod0 = d0[0]; lod1 = d1[0]; if constexpr (TP::on) rec_lo = rc[0]; }
    bool s2 = d0[2] < 0.f && lod0 < d0[2];
    if (s2) { loa = al[2]; lod0 = d0[2]; lod1 = d1[2]; if constexpr (TP::on) rec_lo = rc[2]; }
    bool s3 = hid0 < 0.f || hid0 > d0[1];
    if (s3) { hia = al[1]; hid0 = d0[1]; hid1 = d1[1]; if constexpr (TP::on) rec_hi = rc[1]; }
    bool s4 = d0[2] > 0.f && hid0 > d0[2];
    if (s4) { hia = al[2]; hid0 = d0[2]; hid1 = d1[2]; if constexpr (TP::on) rec_hi = rc[2]; }
    TCOUNT(14, 1, lane);
    if (!(s1 || s2 || s3 || s4)) break;
    lot = tol(loa, lod0, lod1);
    hit = tol(hia, hid0, hid1);
  }
  TCOUNT(15, 1, lane);
  float ac[3] = {0.f, loa, hia}, cost[3];
  TACC(31, tl, lane);
  eval(I3{}, TT{}, ac, cost, nullptr);
  const bool improved = cost[1] < cost[0] || cost[2] < cost[0];
  const float alpha = cost[1] < cost[2] ? loa : hia;
  if constexpr (TP::on) tp.ls_end(improved ? alpha : 0.f, improved ? (cost[1] < cost[2] ? rec_lo : rec_hi) : 0.f, lane);
  return apply(improved ? alpha : 0.f);
}

// tape hooks of the primal kernels: none (every `if constexpr (TP::on)` block compiles away)
struct NoTape {
  static constexpr bool on = false;
};

template <class D, bool G, class TP> PHASE void solver_t(MP m_, LDSA WS<D>* W, Rows<G> R, int lane, TP& tp) {
  MP m = uniform_ptr(m_);
  constexpr int LD = D::LD;
  const int nv = m->nv, nefc = W->nefc;
  const bool newton = m->solver == MJL_SOLVER_NEWTON;
  if (nefc == 0) {
    if (lane < LD) { W->qacc[lane] = W->qacc_ws[lane] = W->qacc_smooth[lane]; W->frc_con[lane] = 0.f; }
    if (lane == 0) { W->niter = 0; W->sc[SC_NACT] = 0.f; }
    SYNC();
    return;
  }
  const float scale = m->scale;
  TSTART(ts);
  // warm start: the cheaper of qacc_warmstart and qacc_smooth. M q and J q (rows < 64) of both
  // candidates with clamped row indices, so every load issues before the first wait; the chosen
  // candidate's M q and J q - aref are kept as Ma and jar (the same values a recompute would give)
  const int mi = lane < nv ? lane : 0, ri = lane < nefc ? lane : 0;
  LDSA float* qc[2] = {W->qacc_ws, W->qacc_smooth};
  float mq[2], jq[2];
#pragma unroll
  for (int w = 0; w < 2; w++) { mq[w] = mrow<D>(W, qc[w], mi); jq[w] = jrow<D>(R.J, qc[w], ri); }
  const float fs = W->frc_smooth[mi], qs = W->qacc_smooth[mi], ar = R.aref[ri], dr = R.D[ri];
  float cost2[2];
#pragma unroll
  for (int w = 0; w < 2; w++) {
    const float g = lane < nv ? 0.5f * (mq[w] - fs) * (qc[w][mi] - qs) : 0.f;
    const float j = jq[w] - ar;
    float c = (lane < nefc && j < 0.f) ? 0.5f * dr * j * j : 0.f;
    for (int r = lane + 64; r < nefc; r += 64) {
      float jr = jrow<D>(R.J, qc[w], r) - R.aref[r];
      if (jr < 0.f) c += 0.5f * R.D[r] * jr * jr;
    }
    cost2[w] = wsum(g + c);
  }
  const int wsel = cost2[0] < cost2[1] ? 0 : 1;
  LDSA float* q0 = qc[wsel];
  if (lane < LD) W->qacc[lane] = q0[lane];
  if (lane < nv) W->Ma[lane] = mq[wsel];
  if (lane < nefc) R.jar[lane] = jq[wsel] - ar;
  for (int r = lane + 64; r < nefc; r += 64) R.jar[r] = jrow<D>(R.J, q0, r) - R.aref[r];
  // (qacc, Ma and jar entries are read next by the lanes that wrote them: no barrier in the primal)
  if constexpr (TP::on) SYNC();
  if constexpr (TP::on) tp.warm(wsel, lane);
  TACC(9, ts, lane);
  // Newton / CG iterations, written so that each helper appears once in the loop body.
  // Exact early exit (Newton): rows are affine in alpha, so if the active set at the new point
  // equals the set the Hessian was built from, no row switched along the step, the cost was one
  // quadratic there and the exact line search landed on its minimiser, where the gradient is
  // zero: the global optimum MuJoCo's tolerance test converges to. In fp32 that test only fires
  // once rounding noise turns the improvement non-positive, which costs extra iterations.
  float cost = 0.f;
  int iter = 0;
  const int maxit = m->iterations;
  const bool exact_exit = newton && nefc <= 256;
  unsigned long long hm[4] = {0ull, 0ull, 0ull, 0ull};
  int nhess = 0, nact = 0;  // Hessians built, active rows summed over them (bench FLOP model)
  auto active_masks = [&](unsigned long long* out) {
#pragma unroll
    for (int c = 0; c < 4; c++) {
      int r = lane + 64 * c;
      out[c] = __ballot(r < nefc && R.jar[r] < 0.f);
    }
  };
  for (bool first = true;; first = false) {
    if (!first) {
      float alpha = solver_linesearch<D, G>(m, W, R, lane, tp);
#ifndef MJL_DIAG_FIXIT
      if (!(alpha != 0.f)) { iter++; break; }  // no improvement: MJX's next cond stops (also on NaN)
#endif
      // (the line search applied the step to qacc, Ma and jar, each entry by the lane that reads it
      // next, so the primal needs no barrier here; the tape's hooks read across lanes)
      if (!newton && lane < nv) { W->gradold[lane] = W->grad[lane]; W->Mgradold[lane] = W->Mgrad[lane]; }
      if constexpr (TP::on) SYNC();
      TACC(10, ts, lane);
    }
    float oldcost = cost, gsq;
    cost = solver_update<D, G>(m, W, R, lane, gsq);
    if constexpr (TP::on) tp.update(W, R, lane);
    if (first && maxit != 1) {  // MJX cond before the first body (iterations == 1 runs one body)
#ifndef MJL_DIAG_FIXIT
      if (maxit <= 0 || scale * sqrtf(gsq) < m->tolerance) break;
#endif
    }
    if (!first) {
      iter++;
      float gnorm = scale * sqrtf(gsq);
      float improvement = scale * (oldcost - cost);
#ifdef MJL_DIAG_FIXIT  // diagnostic: exactly `iterations` iterations (cost attribution by knockouts)
      if (iter >= maxit) break;
      (void)gnorm; (void)improvement;
#else
      if (improvement < m->tolerance || gnorm < m->tolerance || iter >= maxit) break;
#endif
      if (exact_exit) {
        unsigned long long am[4];
        active_masks(am);
#ifndef MJL_DIAG_FIXIT
        if (am[0] == hm[0] && am[1] == hm[1] && am[2] == hm[2] && am[3] == hm[3]) break;
#endif
      }
    }
    TACC(11, ts, lane);
    if (newton) {
      if (exact_exit) {
        active_masks(hm);
        nact += __popcll(hm[0]) + __popcll(hm[1]) + __popcll(hm[2]) + __popcll(hm[3]);
        nhess++;
      }
      float x;
      if constexpr (D::NV < 32) {  // J'DJ goes from the MFMA accumulator straight into the factor's rows
#ifdef MJL_DIAG_KO_HESS
        f32x16 acc = {};
#else
        const f32x16 acc = solver_hessian_acc<D, G>(m, W, R, lane);
#endif
        TACC(12, ts, lane);
#ifdef MJL_DIAG_KO_CHOL
        x = W->grad[lane & 31] + acc[0] * 1e-30f;
#else
        x = chol_aug_factor_solve<D, true>(W->M, W->H, W->invd, nv, W->grad, lane, acc);
#endif
      } else {
        solver_hessian<D, G>(m, W, R, lane);
        TACC(12, ts, lane);
        x = chol_factor_solve<D>(W->H, W->H, W->invd, nv, W->grad, lane);
      }
      TACC(13, ts, lane);  // (Mgrad is CG's: Newton does not store it)
      if constexpr (TP::on) tp.direction(x, 0.f, 0.f, 0.f, lane);
      if (lane < LD) W->search[lane] = (lane < nv) ? -x : 0.f;
    } else {
      float x = chol_solve<D>(W->H, W->invd, lane < nv ? W->grad[lane] : 0.f, lane);  // H holds L(M)
      if (lane < nv) W->Mgrad[lane] = x;
      float num = 0.f, den = 0.f;
      if (!first && lane < nv) {
        num = W->grad[lane] * (x - W->Mgradold[lane]);
        den = W->gradold[lane] * W->Mgradold[lane];
      }
      num = wsum(num);
      den = wsum(den);
      float beta = first ? 0.f : fmaxf(0.f, num / fmaxf(kMinVal, den));  // PR, MJX's floored denominator
      if constexpr (TP::on) tp.direction(x, beta, num, den, lane);
      if (lane < LD) W->search[lane] = (lane < nv) ? -x + beta * W->search[lane] : 0.f;
    }
    SYNC();
  }
  if (lane == 0) { W->niter = iter; W->sc[SC_NACT] = nhess ? (float)nact / (float)nhess : 0.f; }
  // the solution seeds the next solve (MuJoCo mj_fwdConstraint, MJX solver.solve: qacc_warmstart =
  // qacc), so it belongs to forward: a reset's forward leaves the warm start MJX leaves
  if (lane < nv) W->qacc_ws[lane] = W->qacc[lane];
  SYNC();
}
template <class D, bool G> PHASE void solver(MP m_, LDSA WS<D>* W, Rows<G> R, int lane) {
  NoTape nt;
  solver_t<D, G>(m_, W, R, lane, nt);
}

// touch sensors (lane = sensor)   [sensor.sensor_acc, MuJoCo mjSENS_TOUCH]
// Lane = contact: every contact's normal force and ray-box test run in parallel, one wave sum per
// sensor (the sensor loop is uniform, so its constants come through the scalar cache).
template <class D, bool G> PHASE void sensors(MP m_, LDSA WS<D>* W, Rows<G> R, int lane) {
  MP m = uniform_ptr(m_);
  const int ncon = W->ncon, nsensor = m->nsensor;
  for (int c0 = 0; c0 < ncon; c0 += 64) {
    const int c = c0 + lane;
    const bool has = c < ncon;
    int b1 = -1, b2 = -1;
    float fn = 0.f, cp[3] = {0.f, 0.f, 0.f}, cn[3] = {0.f, 0.f, 0.f};
    if (has) {
      typename Rows<G>::F* cr = R.con + c * CONW;
      const int packed = __float_as_int(cr[15]), dim = (packed >> 16) & 0xff;
      b1 = packed & 0xff; b2 = (packed >> 8) & 0xff;
      int nrow = dim == 1 ? 1 : 2 * (dim - 1), r0 = R.con_efc[c];
      for (int r = 0; r < nrow; r++) fn += R.force[r0 + r];
      cp[0] = cr[0]; cp[1] = cr[1]; cp[2] = cr[2];
      cn[0] = cr[3]; cn[1] = cr[4]; cn[2] = cr[5];
    }
    for (int s = 0; s < nsensor; s++) {
      const int site = m->sensor_objid[s], body = m->site_bodyid[site];
      float val = 0.f;
      if (has && fn > 0.f && (b1 == body || b2 == body)) {
        float sg = (b2 == body) ? -1.f : 1.f;
        float dir[3] = {sg * cn[0], sg * cn[1], sg * cn[2]};
        float dp[3] = {cp[0] - W->spos[site][0], cp[1] - W->spos[site][1], cp[2] - W->spos[site][2]};
        float S[9];
        for (int i = 0; i < 9; i++) S[i] = W->smat[site][i];
        float lp[3], lv[3];
        mtv3(lp, S, dp);
        mtv3(lv, S, dir);
        const float sz[3] = {m->site_size[site][0], m->site_size[site][1], m->site_size[site][2]};
        bool hit = false;
        for (int i = 0; i < 3; i++) {  // ray-box test in the site frame (mju_rayGeom, box)
          if (fabsf(lv[i]) <= kMinVal) continue;
          const int i1 = (i + 1) % 3, i2 = (i + 2) % 3;
          for (int side = -1; side <= 1; side += 2) {
            float sol = ((float)side * sz[i] - lp[i]) / lv[i];
            float a = lp[i1] + sol * lv[i1], b = lp[i2] + sol * lv[i2];
            hit |= sol >= 0.f && fabsf(a) <= sz[i1] && fabsf(b) <= sz[i2];
          }
        }
        val = hit ? fn : 0.f;
      }
      val = wsum(val);
      if (lane == 0) W->sens[m->sensor_adr[s]] = (c0 == 0 ? 0.f : W->sens[m->sensor_adr[s]]) + val;
    }
  }
  if (ncon == 0 && lane < nsensor) W->sens[m->sensor_adr[lane]] = 0.f;
  SYNC();
}

// rows that do not fit in LDS: the cold path, kept out of line
// MW: the calling kernel's waves-per-SIMD bound. A callee shared by kernels of different bounds is
// compiled for the loosest, and its register use then caps the tighter kernel's occupancy.
template <class D, int MW = MJL_MINWAVES> NOINL void global_rows_path(MP m, LDSA WS<D>* W, float* scratch_env, int gmax_efc, int gmax_con,
                                               int lane) {
  Rows<true> R = global_rows<D>(scratch_env, gmax_efc, gmax_con);
  build_rows<D, true>(m, W, R, lane);
  solver<D, true>(m, W, R, lane);
  sensors<D, true>(m, W, R, lane);
}

// full forward pass (mjx.forward)
template <class D, int MW = MJL_MINWAVES> PHASE void forward(MP m_, LDSA WS<D>* W, float* scratch_env, int gmax_efc, int gmax_con,
                                      int force_global, int lane, const KinPre& kp) {
  MP m = uniform_ptr(m_);
  constexpr int LD = D::LD;
  STAMP(0, lane);
  kinematics<D>(m, W, lane, kp);
  STAMP(1, lane);
  com_pos_crb<D>(m, W, lane, kp);
  STAMP(2, lane);
  velocity_stage<D>(m, W, lane, kp);
  STAMP(3, lane);
  // factor M into H: qacc_smooth now, CG preconditioner later
  float x = chol_factor_solve<D>(W->M, W->H, W->invd, m->nv, W->frc_smooth, lane);
  if (lane < LD) W->qacc_smooth[lane] = (lane < m->nv) ? x : 0.f;  // first read after build_rows' barriers
  STAMP(4, lane);
  bool ok = false;
  if (!force_global) ok = build_rows<D, false>(m, W, lds_rows<D>(W), lane);
  STAMP(5, lane);
  if (ok) {
    Rows<false> R = lds_rows<D>(W);
    solver<D, false>(m, W, R, lane);
    STAMP(6, lane);
    sensors<D, false>(m, W, R, lane);
    STAMP(7, lane);
  } else {  // more rows than fit in LDS (or forced): this env's slab of global scratch
    global_rows_path<D, MW>(m, W, scratch_env, gmax_efc, gmax_con, lane);
  }
}

// ---------------------------------------------------------------------------------------------
// integration (Euler with eulerdamp / implicitfast)   [forward.euler / forward.implicit]
// ---------------------------------------------------------------------------------------------
template <class D> PHASE void integrate(MP m_, LDSA WS<D>* W, int lane, LDSA float* ap_out = nullptr) {
  MP m = uniform_ptr(m_);
  constexpr int LD = D::LD;
  const int nv = m->nv;
  const float dt = m->timestep;
  // this lane's joint record and dof damping, issued before the first wait
  const JntRec jr = ldrec(&m->jrec[lane < m->njnt ? lane : 0]);
  const float dmp = m->dof_damping[(lane & 31) < nv ? (lane & 31) : 0];
  float qa = (lane < nv) ? W->qacc[lane] : 0.f;
  bool damp = (m->integrator == MJL_INT_IMPLICITFAST || m->eulerdamp) && m->any_damping;
  if (damp) {  // (M + dt*diag(damping)) qacc' = qfrc_smooth + qfrc_constraint
    if constexpr (D::NV < 32) {
      // dt*diag(damping) enters the factor as its MFMA-layout addend (register v of lane l holds
      // row (v&3) + 8(v>>2) + 4(l>>5) of column l&31): no copy of M into H and no barrier for it
      if (lane < nv) W->Mv[lane] = W->frc_smooth[lane] + W->frc_con[lane];  // Mv: solver scratch, free now
      f32x16 C;
      const int c = lane & 31, h = lane >> 5;
#pragma unroll
      for (int v = 0; v < 16; v++) C[v] = ((v & 3) + 8 * (v >> 2) + 4 * h == c && c < nv) ? dt * dmp : 0.f;
      SYNC();
      qa = chol_aug_factor_solve<D, true>(W->M, W->H, W->invd, nv, W->Mv, lane, C);
    } else {
      for (int i = lane; i < D::NV * LD; i += 64) W->H[i] = W->M[i];
      SYNC();
      if (lane < nv) {
        W->H[lane * LD + lane] += dt * dmp;
        W->Mv[lane] = W->frc_smooth[lane] + W->frc_con[lane];
      }
      SYNC();
      qa = chol_factor_solve<D>(W->H, W->H, W->invd, nv, W->Mv, lane);
    }
  }
  if (ap_out && lane < D::LD) ap_out[lane] = (lane < nv) ? qa : 0.f;  // a' for the step adjoint
  if (lane < nv) W->qvel[lane] += dt * qa;
  SYNC();
  if (lane < m->njnt) {
    const int q = jr.qadr, d = jr.dofadr;
    if (jr.isfree) {
      W->qpos[q] += dt * W->qvel[d];
      W->qpos[q + 1] += dt * W->qvel[d + 1];
      W->qpos[q + 2] += dt * W->qvel[d + 2];
      float w[3] = {W->qvel[d + 3], W->qvel[d + 4], W->qvel[d + 5]};
      float nrm = norm3(w);
      float s, c;
      sincosf(0.5f * nrm * dt, &s, &c);
      float qr[4] = {c, w[0] * s, w[1] * s, w[2] * s};
      float qq[4] = {W->qpos[q + 3], W->qpos[q + 4], W->qpos[q + 5], W->qpos[q + 6]};
      qmul(qq, qq, qr);
      qnorm(qq);
      W->qpos[q + 3] = qq[0]; W->qpos[q + 4] = qq[1]; W->qpos[q + 5] = qq[2]; W->qpos[q + 6] = qq[3];
    } else {
      W->qpos[q] += dt * W->qvel[d];
    }
  }
  if (lane == 0) W->sc[SC_TIME] += dt;
  SYNC();
}

// ---------------------------------------------------------------------------------------------
// env wrapper (reference src/envs.py)
// ---------------------------------------------------------------------------------------------
template <class Q> INL void rpy(Q q, float& roll, float& pitch, float& yaw) {  // envs.py:357-365
  float w = q[0], x = q[1], y = q[2], z = q[3];
  roll = atan2f(2.f * (w * x + y * z), 1.f - 2.f * (x * x + y * y));
  pitch = asinf(fminf(fmaxf(2.f * (w * y - z * x), -1.f), 1.f));
  yaw = atan2f(2.f * (w * z + x * y), 1.f - 2.f * (y * y + z * z));
}
template <class P> INL float xydist(float tx, float ty, P p) {
  float dx = tx - p[0], dy = ty - p[1];
  return sqrtf(dx * dx + dy * dy);
}
typedef const CSTA mjlEnvConfig* CP;
template <class S> INL float stance_of(CP c, S sens) {  // envs.py:89-106
  bool r = sens[c->touch_sensor_right_id] > 0.f, l = sens[c->touch_sensor_left_id] > 0.f;
  return (r && l) ? 0.f : ((r && !l) ? 1.f : ((!r && l) ? 2.f : 3.f));
}

// obs entry i of compute_obs (envs.py:317-331): raw obs at index perm[i] (flipped) or i
template <class D> INL float raw_obs(MP m, LDSA WS<D>* W, CP c, int idx) {
  int nj = m->nq - 7;
  if (idx < 4) return W->sc[SC_HEIGHT + idx];  // height, roll, pitch, yaw
  idx -= 4;
  if (idx < nj) return W->qpos[7 + idx];
  idx -= nj;
  if (idx < 6) {  // pelvis-rotation^T applied to the root free-joint linear / angular qvel (envs.py:274-315)
    float R[9];
    q2m(R, W->xquat[c->pelvis_body_id]);
    int h = idx / 3, k = idx % 3;
    return R[k] * W->qvel[3 * h] + R[3 + k] * W->qvel[3 * h + 1] + R[6 + k] * W->qvel[3 * h + 2];
  }
  idx -= 6;
  if (idx < m->nv - 6) return W->qvel[6 + idx];
  idx -= m->nv - 6;
  return W->sc[SC_TF0 + idx];
}
template <class D> INL void write_obs(MP m, LDSA WS<D>* W, CP c, float* obs, int lane) {
  if (lane < c->obs_dim) {
    bool flip = W->sc[SC_FLIP] > 0.5f;
    obs[lane] = flip ? raw_obs<D>(m, W, c, c->obs_perm[lane]) * c->obs_sign[lane] : raw_obs<D>(m, W, c, lane);
  }
}

// threefry2x32-20 (Random123; the generator behind jax.random)
INL uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
INL void threefry2x32(uint32_t k0, uint32_t k1, uint32_t& x0, uint32_t& x1) {
  const uint32_t k2 = k0 ^ k1 ^ 0x1BD11BDAu;
  const uint32_t ks[3] = {k0, k1, k2};
  const int rot[8] = {13, 15, 26, 6, 17, 29, 16, 24};
  x0 += k0; x1 += k1;
#pragma unroll
  for (int i = 0; i < 5; i++) {
#pragma unroll
    for (int j = 0; j < 4; j++) { x0 += x1; x1 = rotl32(x1, rot[(i & 1) * 4 + j]); x1 ^= x0; }
    x0 += ks[(i + 1) % 3];
    x1 += ks[(i + 2) % 3] + (uint32_t)(i + 1);
  }
}
// uniform [0,1) for draw i of env e: key = threefry(seed, counter), bits = threefry(key, (e, i))
INL float uniform01(uint32_t s0, uint32_t s1, uint32_t c0, uint32_t c1, int env, int i) {
  uint32_t k0 = c0, k1 = c1;
  threefry2x32(s0, s1, k0, k1);
  uint32_t x0 = (uint32_t)env, x1 = (uint32_t)i;
  threefry2x32(k0, k1, x0, x1);
  return __uint_as_float((x0 >> 9) | 0x3f800000u) - 1.f;  // jax.random.uniform bit mapping
}

// jax.random on threefry2x32 (jax==0.7.2 `_threefry_split` / `_random_bits` / `_uniform`), for
// resets drawn from per-env JAX keys exactly as single_reset (envs.py:116-147) draws them.
// Partitionable mode (the jax_threefry_partitionable default since jax 0.5): element i of a draw
// or of a split is threefry(key, (0, i)); random bits = x0 ^ x1, a split key = (x0, x1).
// Original mode: a draw of n elements (n padded to even with a 0 count) is threefry(key, (c[j],
// c[j + n'/2])) over c = iota(n), concatenated; split(key, 4) is that draw of 8 words reshaped (4, 2).
INL float jax_bits_to_unit(uint32_t bits) { return __uint_as_float((bits >> 9) | 0x3F800000u) - 1.f; }
INL void jax_split4(int mode, uint32_t k0, uint32_t k1, int j, uint32_t& o0, uint32_t& o1) {
  if (mode == MJL_RNG_JAX_PARTITIONABLE) {
    o0 = 0u; o1 = (uint32_t)j;
    threefry2x32(k0, k1, o0, o1);
  } else {  // words 2j, 2j+1 of threefry over (iota(4), iota(4) + 4)
    uint32_t a0 = (uint32_t)((2 * j) & 3), a1 = a0 + 4u, b0 = a0 + 1u, b1 = b0 + 4u;
    threefry2x32(k0, k1, a0, a1);
    threefry2x32(k0, k1, b0, b1);
    o0 = (2 * j < 4) ? a0 : a1;
    o1 = (2 * j < 4) ? b0 : b1;
  }
}
// element i of jax.random.uniform(key, (n,)) (n = 0 for shape ())
INL float jax_uniform(int mode, uint32_t k0, uint32_t k1, int i, int n) {
  if (mode == MJL_RNG_JAX_PARTITIONABLE) {
    uint32_t x0 = 0u, x1 = (uint32_t)i;
    threefry2x32(k0, k1, x0, x1);
    return jax_bits_to_unit(x0 ^ x1);
  }
  const int np = (n < 1 ? 1 : n) + ((n < 1 ? 1 : n) & 1), h = np / 2;
  auto cnt = [&](int j) { return (uint32_t)(j < (n < 1 ? 1 : n) ? j : 0); };  // iota padded with 0
  const int j = i < h ? i : i - h;
  uint32_t x0 = cnt(j), x1 = cnt(j + h);
  threefry2x32(k0, k1, x0, x1);
  return jax_bits_to_unit(i < h ? x0 : x1);
}

// The launch's KParams as the kernarg segment (the kernels' only argument), through an opaque copy of
// the segment pointer: fields read through it are loaded where they are used (the env step's reset
// runs after the whole step, and a field read in the kernel prologue would hold an SGPR across it).
// Kernel bodies only: in a called function the intrinsic is not the kernel's segment (it lowers to a
// null pointer), so a callee takes the pointer as an argument.
// Guarded two ways: the debug build (make debug, -DMJL_DEBUG) traps on a null pointer, and
// tests/test_kernarg_guard.py scans the shipped code object for a non-kernel function that loads
// through a zeroed SGPR pair (the round-5 fault: `s_mov_b64 s[4:5], 0` feeding the loads).
INL const CSTA KParams* kparams_late() {
  const CSTA KParams* p = (const CSTA KParams*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
#ifdef MJL_DEBUG
  if (p == nullptr) __builtin_trap();
#endif
  return p;
}

// single_reset (envs.py:115-202): random pose / velocity, forward, target, aux, obs. Out of line, and it
// reads the launch's arguments itself through P (the caller's kparams_late() at the call): the caller
// keeps none of them live across the step (round 4 passed ~14 of them by value, which raised the
// env-step kernel's SGPR spills 152 -> 178).
template <class D, int MW = MJL_MINWAVES> NOINL void env_reset(MP m_, LDSA WS<D>* W, const CSTA KParams* P, int env,
                                                                int lane, LDSA float* aux_out, float* obs_out) {
  MP m = uniform_ptr(m_);
  struct {
    const mjlEnvConfig* cfg;
    const float* noise;
    float* scratch_env;
    int gmax_efc, gmax_con, force_global;
    uint32_t s0, s1, c0, c1;
    const uint32_t* keys;  // per-env jax.random keys [nenv, 2] (key mode) or null
    int key_mode;
  } A;
  A.cfg = P->env; A.noise = P->noise;
  A.scratch_env = P->scratch + (size_t)env * (size_t)P->scratch_stride;
  A.gmax_efc = P->gmax_efc; A.gmax_con = P->gmax_con; A.force_global = P->force_global_rows;
  A.s0 = P->seed_lo; A.s1 = P->seed_hi; A.keys = P->keys; A.key_mode = P->key_mode;
  {  // RNG counter = launch counter + the batch's device counter base (hipGraph replays)
    const unsigned long long c = ((unsigned long long)P->ctr_hi << 32 | P->ctr_lo) + (P->ctr_base ? *P->ctr_base : 0ull);
    A.c0 = (uint32_t)c; A.c1 = (uint32_t)(c >> 32);
  }
  CP c = (CP)A.cfg;
  const int nj = m->nq - 7, nv = m->nv, nd = nj + nv + 2;
  float u = 0.f;
  if (lane < nd) {
    if (A.noise) {
      u = A.noise[(size_t)env * nd + lane];
    } else if (A.keys) {  // k1..k4 = split(key, 4); uniform(k1, (nq-7,)), uniform(k2, (nv,)), bernoulli(k3), uniform(k4)
      const int which = lane < nj ? 0 : lane < nj + nv ? 1 : lane == nj + nv ? 2 : 3;
      const int idx = which == 0 ? lane : which == 1 ? lane - nj : 0;
      const int n = which == 0 ? nj : which == 1 ? nv : 0;
      uint32_t s0, s1;
      jax_split4(A.key_mode, A.keys[2 * (size_t)env], A.keys[2 * (size_t)env + 1], which, s0, s1);
      u = jax_uniform(A.key_mode, s0, s1, idx, n);
    } else {
      u = uniform01(A.s0, A.s1, A.c0, A.c1, env, lane);
    }
  }
  const KinPre kp = kin_prefetch(m, lane);
  if (lane < m->nq) W->qpos[lane] = m->qpos0[lane];
  if (lane < 32) W->ctrl[lane] = 0.f;
  if (lane < D::LD) { W->qacc_ws[lane] = 0.f; W->qvel[lane] = 0.f; }
  SYNC();
  if (lane < nj) W->qpos[7 + lane] += c->random_joint_noise * (u * 2.f - 1.f);
  if (lane >= nj && lane < nj + nv) W->qvel[lane - nj] = c->random_vel_noise * (u * 2.f - 1.f);
  float uflip = rdlane(u, nj + nv), uspeed = rdlane(u, nj + nv + 1);
  if (lane == 0) {
    W->sc[SC_FLIP] = c->random_flip ? (uflip < 0.5f ? 1.f : 0.f) : 0.f;
    W->sc[SC_TIME] = 0.f;
  }
  SYNC();
  if (c->initial_velocity_max > 0.f) {
    kinematics<D>(m, W, lane, kp);  // the first forward's pelvis position (positions depend on qpos only)
    LDSA float* bp = W->xpos[c->pelvis_body_id];
    float tx = bp[0] + c->target_dist, ty = bp[1];
    float dx = tx - bp[0], dy = ty - bp[1];
    float dxy = sqrtf(dx * dx + dy * dy);
    float vmag = uspeed * c->initial_velocity_max;
    float vx = dxy > 1e-6f ? vmag * dx / dxy : 0.f;
    float vy = dxy > 1e-6f ? vmag * dy / dxy : 0.f;
    SYNC();
    if (lane == 0) { W->qvel[0] = vx; W->qvel[1] = vy; }
    SYNC();
  }
  forward<D, MW>(m, W, A.scratch_env, A.gmax_efc, A.gmax_con, A.force_global, lane, kp);
  if (lane == 0) {
    LDSA float* bp = W->xpos[c->pelvis_body_id];
    float tx = bp[0] + c->target_dist, ty = bp[1], tz = bp[2];
    float dxp = tx - bp[0], dyp = ty - bp[1];
    float dist = fmaxf(xydist(tx, ty, bp), xydist(tx, ty, W->xpos[c->head_body_id]));
    float roll, pitch, yaw;
    rpy(W->xquat[c->pelvis_body_id], roll, pitch, yaw);
    float angle = atan2f(dyp, dxp) - yaw;
    float soft = dist / (1.f + fabsf(dist));
    float sa, ca;
    sincosf(angle, &sa, &ca);
    W->sc[SC_HEIGHT] = bp[2]; W->sc[SC_ROLL] = roll; W->sc[SC_PITCH] = pitch; W->sc[SC_YAW] = yaw;
    W->sc[SC_TF0] = soft * sa; W->sc[SC_TF1] = soft * ca;
    float a[MJL_AUX_DIM] = {W->sc[SC_FLIP], tx, ty, tz, 0.f, stance_of(c, W->sens), 0.f, -dist / m->timestep, 0.f};
    for (int i = 0; i < MJL_AUX_DIM; i++) aux_out[i] = a[i];
  }
  SYNC();
  if (obs_out) write_obs<D>(m, W, c, obs_out, lane);
}

// post-step part of single_step (envs.py:347-492): reward, termination, aux, obs
// (skip_done_obs: finished envs' observations are replaced by the auto-reset's, so not written)
template <class D> PHASE void env_post(MP m_, LDSA WS<D>* W, const mjlEnvConfig* cfg, LDSA float* aux, float* obs,
                                       int lane, bool skip_done_obs) {
  MP m = uniform_ptr(m_);
  CP c = (CP)cfg;
  float pw = 0.f, st = 0.f;  // energy terms over the actuated hinge dofs (mean over nv - 6)
  if (lane >= 6 && lane < m->nv) {
    float fa = W->frc_act[lane];
    pw = fabsf(fa * W->qvel[lane]);
    st = fa * fa;
  }
  pw = wsum(pw);
  st = wsum(st);
  if (lane == 0) {
    const float dt = m->timestep;
    LDSA float* hp = W->xpos[c->head_body_id];
    LDSA float* bp = W->xpos[c->pelvis_body_id];
    float height = bp[2];
    float roll, pitch, yaw;
    rpy(W->xquat[c->pelvis_body_id], roll, pitch, yaw);
    float tx = aux[1], ty = aux[2], tz = aux[3];
    float dist = fmaxf(xydist(tx, ty, bp), xydist(tx, ty, hp));
    float progress = (-dist / dt - aux[7]) * c->progress_weight;
    float nj = (float)(m->nv - 6);
    float energy = c->electricity_cost * (pw / nj) + c->stall_torque_cost * (st / nj);
    float posture = ((pitch > -0.087f) && (pitch < 0.174f)) ? 0.f : fabsf(pitch);
    posture += ((roll > -0.174f) && (roll < 0.174f)) ? 0.f : fabsf(roll);
    posture *= c->posture_penalty_weight;
    float tall = c->tall_bonus_weight * (height > c->tall_height_threshold ? 1.f : -1.f);
    float time = W->sc[SC_TIME];
    float old_st = aux[5], st_time = aux[6];
    float new_st = stance_of(c, W->sens);
    bool changed = new_st != old_st;
    float dur = time - st_time;
    float stance_rew = (changed && dur > 0.1f) ? c->stance_time_reward_weight * dur / dt : 0.f;
    float st_upd = changed ? new_st : old_st;
    float st_time_upd = changed ? time : st_time;
    bool close = dist < c->target_threshold;
    float close_count = close ? aux[4] + 1.f : 0.f;
    float bonus = close ? 2.f : 0.f;
    if (close_count >= (float)c->stop_frames) { tx = bp[0] + c->target_dist; ty = bp[1]; tz = bp[2]; close_count = 0.f; }
    float dxp = tx - bp[0], dyp = ty - bp[1];
    float dist2 = fmaxf(xydist(tx, ty, bp), xydist(tx, ty, hp));
    float angle = atan2f(dyp, dxp) - yaw;
    float soft = dist2 / (1.f + fabsf(dist2));
    float sa, ca;
    sincosf(angle, &sa, &ca);
    float reward = progress + bonus + stance_rew - energy + tall - posture;
    float ep = aux[8] + 1.f;
    bool fallen = height < c->terminate_height;
    float term = fallen ? 1.f : 0.f;
    float trunc = (c->max_episode_steps > 0 && ep >= (float)c->max_episode_steps) ? 1.f : 0.f;
    if (fallen) reward += c->terminate_reward;
    W->sc[SC_REW] = reward; W->sc[SC_TERM] = term; W->sc[SC_TRUNC] = trunc; W->sc[SC_DONE] = fmaxf(term, trunc);
    W->sc[SC_HEIGHT] = height; W->sc[SC_ROLL] = roll; W->sc[SC_PITCH] = pitch; W->sc[SC_YAW] = yaw;
    W->sc[SC_TF0] = soft * sa; W->sc[SC_TF1] = soft * ca;
    float a[MJL_AUX_DIM] = {aux[0], tx, ty, tz, close_count, st_upd, st_time_upd, -dist2 / dt, ep};
    for (int i = 0; i < MJL_AUX_DIM; i++) aux[i] = a[i];
  }
  SYNC();
  if (!(skip_done_obs && W->sc[SC_DONE] > 0.5f)) write_obs<D>(m, W, c, obs, lane);
}

// merge a pooled reset (mjl_env_fill_reset_pool, row = slot * nenv + env) into the wave: the
// state, aux, observation and (store_derived) the derived fields an in-place env_reset leaves
template <class D> INL void rs_load(MP m, const CSTA KParams* Pk, LDSA WS<D>* W, LDSA float* aux, float* obs,
                                    size_t env, int lane) {
  const CSTA KParams& P = *Pk;
  const CSTA StateBuf& R = P.rs;
  const int nq = m->nq, nv = m->nv, nu = m->nu, nb = m->nbody;
  if (lane < nq) W->qpos[lane] = R.qpos[(size_t)env * nq + lane];
  if (lane < nv) {
    const size_t o = (size_t)env * nv + lane;
    W->qvel[lane] = R.qvel[o]; W->qacc_ws[lane] = R.qacc_warmstart[o];
    if (P.store_derived) {
      W->qacc[lane] = R.qacc[o]; W->frc_act[lane] = R.qfrc_actuator[o]; W->frc_bias[lane] = R.qfrc_bias[o];
      W->frc_passive[lane] = R.qfrc_passive[o]; W->frc_con[lane] = R.qfrc_constraint[o];
      W->qacc_smooth[lane] = R.qacc_smooth[o];
    }
  }
  if (lane < nu) W->ctrl[lane] = R.ctrl[(size_t)env * nu + lane];
  if (lane < MJL_AUX_DIM) aux[lane] = R.aux[(size_t)env * MJL_AUX_DIM + lane];
  const int od = P.env->obs_dim;
  if (lane < od) obs[lane] = P.rs_obs[(size_t)env * od + lane];
  if (P.store_derived) {
    for (int i = lane; i < nb * 3; i += 64) W->xpos[i / 3][i % 3] = R.xpos[(size_t)env * nb * 3 + i];
    for (int i = lane; i < nb * 4; i += 64) W->xquat[i / 4][i % 4] = R.xquat[(size_t)env * nb * 4 + i];
    if (lane < m->nsensordata) W->sens[lane] = R.sensordata[(size_t)env * m->nsensordata + lane];
  }
  if (lane == 0) {
    W->sc[SC_TIME] = R.time[env];
    W->sc[SC_HEIGHT] = R.stats[(size_t)env * 4 + 3];  // a pool slot keeps the pelvis height there
    if (P.store_derived) {
      W->ncon = (int)R.stats[(size_t)env * 4 + 0];
      W->nefc = (int)R.stats[(size_t)env * 4 + 1];
      W->niter = (int)R.stats[(size_t)env * 4 + 2];
    }
  }
  SYNC();
}

// ---------------------------------------------------------------------------------------------
// the kernel: one workgroup (= one wavefront) per env
// ---------------------------------------------------------------------------------------------
// MW = the waves-per-SIMD bound of the launch: 2 (the full-occupancy launches: 2048 envs resident on
// 256 CUs) or 1 (launches of at most one wave per SIMD, e.g. C3's 1024-env rollout). The one-wave
// instantiation does not take the whole 512-entry register file: it compiles to the same 248 VGPRs (+ 32
// AGPRs) with fewer SGPR spills (69 against 94 in the env step); its gain is the compiler's schedule and
// spill placement under the looser bound, not registers.
template <class D, int MODE, int MW = MJL_MINWAVES> __global__ __launch_bounds__(64, MW) void step_kernel(KParams P) {
  __shared__ WS<D> Ws;
  __shared__ float aux_s[MJL_AUX_DIM + 3];
  LDSA WS<D>* W = (LDSA WS<D>*)&Ws;
  LDSA float* aux = (LDSA float*)aux_s;
  constexpr int LD = D::LD;
  MP m = (MP)P.m;
  const int env = block_env();
  const int lane = threadIdx.x;
  if (env >= P.nenv) return;
  if ((MODE == MODE_FORWARD || MODE == MODE_ENV_RESET) && P.mask && !(P.mask[env] > 0.5f)) return;
  if (MODE == MODE_ENV_RESET && P.pool_slot >= 0) {  // reset-pool fill: slot pool_slot of this env
    const int n = min(*P.pool_n, P.pool_slots);
    if (P.pool_slot == 0 && lane == 0) { P.pool_ctl[2 * env] = 0; P.pool_ctl[2 * env + 1] = n; }
    if (P.pool_slot >= n) return;
  }
  STAMP(36, lane);
  const int nq = m->nq, nv = m->nv, nu = m->nu;
  const StateBuf& S = P.s;
  float* const scratch_env = P.scratch + (size_t)env * (size_t)P.scratch_stride;
  // vectors beyond nv must read as zero in the LD-wide row kernels
  for (int i = lane; i < LD; i += 64) {
    W->qvel[i] = 0.f; W->qacc_ws[i] = 0.f;
    W->frc_bias[i] = W->frc_passive[i] = W->frc_act[i] = W->frc_smooth[i] = W->qacc_smooth[i] = 0.f;
    W->qacc[i] = W->frc_con[i] = W->grad[i] = W->Mgrad[i] = W->search[i] = W->Ma[i] = W->Mv[i] = 0.f;
    W->gradold[i] = W->Mgradold[i] = 0.f;
  }
  SYNC();

  if (MODE == MODE_ENV_RESET) {
    env_reset<D, MW>(m, W, kparams_late(), env, lane, aux, P.obs ? P.obs + (size_t)env * P.env->obs_dim : nullptr);
  } else {
    const KinPre kp = kin_prefetch(m, lane);  // issued before the state loads: the latencies overlap
    if (MODE == MODE_SPEEDTEST) {  // fresh make_data, qvel[0] = vel (mjx_humanoid_speed_test.py:50-55)
      if (lane < nq) W->qpos[lane] = m->qpos0[lane];
      if (lane < nv) W->qvel[lane] = (lane == 0) ? P.vel[env] : 0.f;
      if (lane < nu) W->ctrl[lane] = 0.f;
      if (lane == 0) W->sc[SC_TIME] = 0.f;
    } else {
      // every state load issues before the first wait: clamped lane indices instead of a branch around
      // each load (each branch waited for its own load: ~7 dependent HBM round trips per env step)
      // (a zero-size field clamps to index 0 and is not read: no load before a user buffer's start)
      const int iq = lane < nq ? lane : max(nq - 1, 0), iv = lane < nv ? lane : max(nv - 1, 0);
      const int iu = lane < nu ? lane : max(nu - 1, 0);
      const float q = nq > 0 ? S.qpos[(size_t)env * nq + iq] : 0.f;
      const float v = nv > 0 ? S.qvel[(size_t)env * nv + iv] : 0.f;
      const float w = nv > 0 ? S.qacc_warmstart[(size_t)env * nv + iv] : 0.f;
      const float* csrc = (MODE == MODE_ENV_STEP || (MODE == MODE_STEP && P.in_ctrl)) ? P.in_ctrl : S.ctrl;
      float c = nu > 0 ? csrc[(size_t)env * nu + iu] : 0.f;
      const float t = S.time[env];
      float ax = 0.f, sgn = 1.f;
      int perm = iu;
      if (MODE == MODE_ENV_STEP) {
        const int ia = lane < MJL_AUX_DIM ? lane : MJL_AUX_DIM - 1;
        ax = S.aux[(size_t)env * MJL_AUX_DIM + ia];
        perm = nu > 0 ? P.env->act_perm[iu] : 0;
        sgn = nu > 0 ? P.env->act_sign[iu] : 1.f;
      }
      if (lane < nq) W->qpos[lane] = q;
      if (lane < nv) { W->qvel[lane] = v; W->qacc_ws[lane] = w; }
      if (lane == 0) W->sc[SC_TIME] = t;
      if (MODE == MODE_ENV_STEP) {  // flip + clip the action (envs.py:335-344): act[perm[j]] from lane perm[j]
        if (lane < MJL_AUX_DIM) aux[lane] = ax;
        const bool flip = rdlane(ax, 0) > 0.5f;
        const float ap = __shfl(c, perm);
        c = fminf(fmaxf(flip ? ap * sgn : c, -1.f), 1.f);
        if (lane == 0) W->sc[SC_FLIP] = ax;
      }
      if (lane < nu) W->ctrl[lane] = c;
    }
    SYNC();
    forward<D, MW>(m, W, scratch_env, P.gmax_efc, P.gmax_con, P.force_global_rows, lane, kp);
    if (MODE != MODE_FORWARD) integrate<D>(m, W, lane);
    STAMP(8, lane);
    const CSTA KParams& P = *kparams_late();  // the tail's arguments, loaded here (see kparams_late)
    if (MODE == MODE_ENV_STEP) {
      float* obs = P.obs + (size_t)env * P.env->obs_dim;
      env_post<D>(m, W, P.env, aux, obs, lane, P.auto_reset != 0);
      STAMP(37, lane);
      if (lane == 0) { P.rew[env] = W->sc[SC_REW]; P.term[env] = W->sc[SC_TERM]; P.trunc[env] = W->sc[SC_TRUNC]; }
      bool bad = (lane < nq && !isfinite(W->qpos[lane])) || (lane < nv && !isfinite(W->qvel[lane]));
      bool anybad = __ballot(bad) != 0ull;
      if (lane == 0) W->sc[SC_NAN] = anybad ? 1.f : 0.f;
      SYNC();
      if (P.auto_reset && W->sc[SC_DONE] > 0.5f) {  // merge_if_done (train_ppo.py:154-161)
        int slot = -1;  // the env's next pooled reset, if one is left (key-drawn resets are never pooled)
        if (P.pool_ctl && !P.keys) {
          const int cur = P.pool_ctl[2 * env], lim = P.pool_ctl[2 * env + 1];
          slot = __builtin_amdgcn_readfirstlane(cur < lim ? cur : -1);
        }
        if (slot >= 0) {
          rs_load<D>(m, &P, W, aux, obs, (size_t)slot * P.nenv + env, lane);
          if (lane == 0) P.pool_ctl[2 * env] = slot + 1;
        } else {
          env_reset<D, MW>(m, W, kparams_late(), env, lane, aux, obs);
        }
      }
      STAMP(38, lane);
    }
  }
  SYNC();
  {  // ---- write back (the launch's arguments loaded here, see kparams_late)
  const CSTA KParams& P = *kparams_late();
  const CSTA StateBuf& S = P.s;
  if (MODE == MODE_SPEEDTEST) {
    if (lane == 0) P.out_speed[env] = W->qpos[0];
    return;
  }
  if (MODE == MODE_FORWARD && lane < nv) S.qacc_warmstart[(size_t)env * nv + lane] = W->qacc_ws[lane];
  if (MODE != MODE_FORWARD) {
    if (lane < nq) S.qpos[(size_t)env * nq + lane] = W->qpos[lane];
    if (lane < nv) {
      S.qvel[(size_t)env * nv + lane] = W->qvel[lane];
      S.qacc_warmstart[(size_t)env * nv + lane] = W->qacc_ws[lane];
    }
    if (lane < nu) S.ctrl[(size_t)env * nu + lane] = W->ctrl[lane];
    if (lane == 0) S.time[env] = W->sc[SC_TIME];
    if ((MODE == MODE_ENV_STEP || MODE == MODE_ENV_RESET) && lane < MJL_AUX_DIM)
      S.aux[(size_t)env * MJL_AUX_DIM + lane] = aux[lane];
  }
  if (MODE == MODE_FORWARD || P.store_derived) {
    if (lane < nv) {
      size_t o = (size_t)env * nv + lane;
      S.qacc[o] = W->qacc[lane]; S.qfrc_actuator[o] = W->frc_act[lane]; S.qfrc_bias[o] = W->frc_bias[lane];
      S.qfrc_passive[o] = W->frc_passive[lane]; S.qfrc_constraint[o] = W->frc_con[lane];
      S.qacc_smooth[o] = W->qacc_smooth[lane];
    }
    const int nb = m->nbody;
    for (int i = lane; i < nb * 3; i += 64) S.xpos[(size_t)env * nb * 3 + i] = W->xpos[i / 3][i % 3];
    for (int i = lane; i < nb * 4; i += 64) S.xquat[(size_t)env * nb * 4 + i] = W->xquat[i / 4][i % 4];
    if (lane < m->nsensordata) S.sensordata[(size_t)env * m->nsensordata + lane] = W->sens[lane];
    if (lane == 0) {
      S.stats[(size_t)env * 4 + 0] = (float)W->ncon;
      S.stats[(size_t)env * 4 + 1] = (float)W->nefc;
      S.stats[(size_t)env * 4 + 2] = (float)W->niter;
      S.stats[(size_t)env * 4 + 3] = (MODE == MODE_ENV_STEP) ? W->sc[SC_NAN] : W->sc[SC_NACT];
    }
  }
  if (MODE == MODE_ENV_RESET && P.pool_slot >= 0 && lane == 0) S.stats[(size_t)env * 4 + 3] = W->sc[SC_HEIGHT];
  }
  STAMP(39, lane);
}

}  // namespace mjl
