// Reverse-mode derivative (VJP) of one mjx.step and of one env step, for APG
// (reference train_apg.py:161-209 differentiates the discounted return through mjx.step).
//
// One wave per env, like the forward kernel: the step is recomputed in LDS (per-step remat, as
// train_apg.py:187-189 checkpoints every step), then the reverse passes run phase by phase.
// Derivative conventions (DESIGN.md "APG"):
//  * implicit mode (default): the constraint solve is differentiated at its converged active set A
//    (implicit function): qacc = Hc^-1 (qfrc_smooth + J_A' D_A aref_A), Hc = M + J_A' D_A J_A; and
//    the total force that enters the integrator, qfrc_smooth + J' f, equals M qacc there;
//  * unrolled mode (MJL_OPT_VJP_UNROLLED): the solve's iterations as executed are differentiated,
//    branch decisions fixed (what jax.grad through MJX's fixed-count solver computes; the reference
//    APG runs CG 4/4, train_apg.py:101-105,187-189): the recompute records a tape (SolveTape) and
//    adj_solver_unrolled sweeps it backwards (algorithm: tests/unrolled_solver_ref.py); the
//    integrator's force is qfrc_smooth + qfrc_constraint of the stopped solve, as forward.py has it;
//  * qacc_warmstart only seeds the solver and gets no cotangent;
//  * piecewise-constant quantities (contact/limit activity, target jumps, flags) follow the branch
//    the primal takes, as reverse-mode autodiff of the reference does.
// Checked against the exact Jacobian of the fp64 oracle (oracle/dual.hpp) in tests/test_adjoint.py.

#include "apg_kernels.hip"  // ApgPostArgs / apg_post_wave (the APG record's fused post-step update)

namespace mjl {

// ------------------------------------------------------------------- derivative helpers
INL void add3(float* a, const float* b) { a[0] += b[0]; a[1] += b[1]; a[2] += b[2]; }
// r = a x b  ->  abar += b x rbar, bbar += rbar x a
template <class A, class B> INL void cross3_adj(A a, B b, const float* rb, float* ab, float* bb) {
  float t[3];
  cross3(t, b, rb); add3(ab, t);
  cross3(t, rb, a); add3(bb, t);
}
// r = a (x) b (quaternion product)
template <class A, class B> INL void qmul_adj(A a, B b, const float* r, float* ab, float* bb) {
  bb[0] += a[0] * r[0] + a[1] * r[1] + a[2] * r[2] + a[3] * r[3];
  bb[1] += -a[1] * r[0] + a[0] * r[1] + a[3] * r[2] - a[2] * r[3];
  bb[2] += -a[2] * r[0] - a[3] * r[1] + a[0] * r[2] + a[1] * r[3];
  bb[3] += -a[3] * r[0] + a[2] * r[1] - a[1] * r[2] + a[0] * r[3];
  ab[0] += b[0] * r[0] + b[1] * r[1] + b[2] * r[2] + b[3] * r[3];
  ab[1] += -b[1] * r[0] + b[0] * r[1] - b[3] * r[2] + b[2] * r[3];
  ab[2] += -b[2] * r[0] + b[3] * r[1] + b[0] * r[2] - b[1] * r[3];
  ab[3] += -b[3] * r[0] - b[2] * r[1] + b[1] * r[2] + b[0] * r[3];
}
// m = q2m(q)
template <class Q, class MB> INL void q2m_adj(Q q, MB mb, float* qb) {
  const float w = q[0], x = q[1], y = q[2], z = q[3];
  qb[0] += 2.f * (-z * mb[1] + y * mb[2] + z * mb[3] - x * mb[5] - y * mb[6] + x * mb[7]);
  qb[1] += 2.f * (y * mb[1] + z * mb[2] + y * mb[3] - 2.f * x * mb[4] - w * mb[5] + z * mb[6] + w * mb[7] - 2.f * x * mb[8]);
  qb[2] += 2.f * (-2.f * y * mb[0] + x * mb[1] + w * mb[2] + x * mb[3] + z * mb[5] - w * mb[6] + z * mb[7] - 2.f * y * mb[8]);
  qb[3] += 2.f * (-2.f * z * mb[0] - w * mb[1] + x * mb[2] + w * mb[3] - 2.f * z * mb[4] + y * mb[5] + x * mb[6] + y * mb[7]);
}
// q = p / |p| (qnorm): pbar += (qbar - q (q . qbar)) / |p|
INL void qnorm_adj(const float* p, const float* qb, float* pb) {
  float n = sqrtf(p[0] * p[0] + p[1] * p[1] + p[2] * p[2] + p[3] * p[3]);
  if (n < kMinVal) return;
  float inv = 1.f / n, q[4] = {p[0] * inv, p[1] * inv, p[2] * inv, p[3] * inv};
  float d = q[0] * qb[0] + q[1] * qb[1] + q[2] * qb[2] + q[3] * qb[3];
  for (int i = 0; i < 4; i++) pb[i] += (qb[i] - q[i] * d) * inv;
}
// r = m v (row-major 3x3)
template <class M, class V> INL void mv3_adj(M m, V v, const float* rb, float* mb, float* vb) {
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) { mb[3 * i + j] += rb[i] * v[j]; vb[j] += m[3 * i + j] * rb[i]; }
}
// u = v / |v| with the forward's norm3 (normalize_with_norm)
INL void norm3_adj(const float* v, const float* ub, float* vb) {
  float n = sqrtf(dot3(v, v));
  float inv = 1.f / (n + (n == 0.f ? 1e-6f : 0.f));
  float u[3] = {v[0] * inv, v[1] * inv, v[2] * inv};
  float d = dot3(u, ub);
  for (int i = 0; i < 3; i++) vb[i] += (ub[i] - u[i] * d) * inv;
}
template <class V, class U> INL void cross_motion_adj(V v, U u, const float* rb, float* vb, float* ub) {
  cross3_adj(v, u, rb, vb, ub);              // r_ang = v_a x u_a
  cross3_adj(v, u + 3, rb + 3, vb, ub + 3);  // r_lin += v_a x u_l
  cross3_adj(v + 3, u, rb + 3, vb + 3, ub);  // r_lin += v_l x u_a
}
template <class V, class F> INL void cross_force_adj(V v, F f, const float* rb, float* vb, float* fb) {
  cross3_adj(v, f, rb, vb, fb);                  // r_ang = v_a x f_a
  cross3_adj(v + 3, f + 3, rb, vb + 3, fb + 3);  //       + v_l x f_l
  cross3_adj(v, f + 3, rb + 3, vb, fb + 3);      // r_lin = v_a x f_l
}
// r = I(i) v (inert_vec): vbar += I rbar (I symmetric), ibar += dr/di . rbar
template <class I, class V> INL void inert_vec_adj(I i, V v, const float* rb, float* ib, float* vb) {
  if (vb) {
    float t[6];
    inert_vec(t, i, rb);
    for (int k = 0; k < 6; k++) vb[k] += t[k];
  }
  if (ib) {
    ib[0] += rb[0] * v[0]; ib[1] += rb[1] * v[1]; ib[2] += rb[2] * v[2];
    ib[3] += rb[0] * v[1] + rb[1] * v[0]; ib[4] += rb[0] * v[2] + rb[2] * v[0]; ib[5] += rb[1] * v[2] + rb[2] * v[1];
    ib[6] += -rb[1] * v[5] + rb[2] * v[4] + rb[4] * v[2] - rb[5] * v[1];
    ib[7] += rb[0] * v[5] - rb[2] * v[3] - rb[3] * v[2] + rb[5] * v[0];
    ib[8] += -rb[0] * v[4] + rb[1] * v[3] + rb[3] * v[1] - rb[4] * v[0];
    ib[9] += rb[3] * v[3] + rb[4] * v[4] + rb[5] * v[5];
  }
}
// impedance with its derivative d imp / d pos (kbi; power 2 and general power)
INL float imp_dpos(const CSTA float* solimp, float pos) {
  float dmin = fminf(fmaxf(solimp[0], kMinImp), kMaxImp);
  float dmax = fminf(fmaxf(solimp[1], kMinImp), kMaxImp);
  float width = fmaxf(kMinVal, solimp[2]);
  float mid = fminf(fmaxf(solimp[3], kMinImp), kMaxImp);
  float power = fmaxf(1.f, solimp[4]);
  float x = fabsf(pos) / width;
  if (x > 1.f) return 0.f;
  float y, dy;
  if (power == 2.f) {
    y = (x < mid) ? (1.f / mid) * x * x : 1.f - (1.f / (1.f - mid)) * (1.f - x) * (1.f - x);
    dy = (x < mid) ? 2.f * x / mid : 2.f * (1.f - x) / (1.f - mid);
  } else {
    y = (x < mid) ? (1.f / powf(mid, power - 1.f)) * powf(x, power)
                  : 1.f - (1.f / powf(1.f - mid, power - 1.f)) * powf(1.f - x, power);
    dy = (x < mid) ? power / powf(mid, power - 1.f) * powf(x, power - 1.f)
                   : power / powf(1.f - mid, power - 1.f) * powf(1.f - x, power - 1.f);
  }
  float imp = dmin + y * (dmax - dmin);
  if (imp < dmin || imp > dmax) return 0.f;
  return (dmax - dmin) * dy * (pos < 0.f ? -1.f : 1.f) / width;
}

// ------------------------------------------------------------------- adjoint workspace (LDS)
// WSA_P1..P3: the adjoint workspace around its dense arrays (Lc, invdc: the factor of Hc; Mb: the
// cotangent of M; uv: unrolled-mode staging). WSAL<DM> (lean replay) drops them: it reads Lc / invdc
// from the tape slot and forms M-bar from its rank-one terms (adj_mass), so the replay fits the
// 20 KB / 8-waves-per-CU LDS budget with WSB.
#define WSA_P1                                                                                       \
  static constexpr int NV = DM::NV, LD = DM::LD, NB = DM::NB, NJ = DM::NJ, NG = DM::NG;             \
  /* forward values kept for the reverse passes */                                                 \
  float qpos0[MJL_MAXQ], qvel0[LD];    /* pre-step state */                                        \
  alignas(16) float mq[LD][4];         /* lean mass reverse: (mu, rb, qacc, a') per dof */
#define WSA_P2                                                                                       \
  float ap[LD];                        /* integrator acceleration a' */                            \
  float lp[NB][3], lq[NB][4];          /* body transform in the parent frame */                    \
  float ftmp[NV][6];                   /* scratch: f_i = I(crb) cdof_i, then its cotangent */      \
  /* cotangents */                                                                                 \
  float qposb[MJL_MAXQ], qvelb[LD], ctrlb[MJL_MAXU], auxb[MJL_AUX_DIM + 3];                        \
  float frcsb[LD], qaccb[LD], frcactb[LD], mu[LD], rb[LD], vtmp[LD];                               \
  float xposb[NB][3], xquatb[NB][4], xmatb[NB][9], xiposb[NB][3], scomb[NB][3];                    \
  float xanchorb[NJ][3], xaxisb[NJ][3], gposb[NG][3], gaxisb[NG][3];                               \
  float cdofb[NV][6], cinertb[NB][10], crbb[NB][10], cvelb[NB][6], caccb[NB][6], cfrcb[NB][6], cfsubb[NB][6]; \
  float Sb[NB][6], Ub[NB][6], Tb[NB][6];
#define WSA_P3                                                                                       \
  float qfcb[LD];                      /* unrolled mode: cotangent of the final qfrc_constraint */ \
  float wsb[LD];                       /* unrolled mode: cotangent of the input qacc_warmstart */
template <class DM> struct WSA {
  WSA_P1
  alignas(16) float Lc[NV * LD];       // factor of Hc at the converged active set
  alignas(16) float invdc[LD];
  WSA_P2
  alignas(16) float Mb[NV * LD];
  WSA_P3
  alignas(16) float uv[3][LD];         // unrolled mode: vectors staged for M v / J v products
};
template <class DM> struct WSAL {  // lean replay: WSA without Lc, invdc, Mb
  WSA_P1
  WSA_P2
  WSA_P3
  alignas(16) float uv[3][LD];         // unrolled mode: vectors staged for M v / J v products
};
template <class AT> struct is_lean { static constexpr bool value = false; };
template <class DM> struct is_lean<WSAL<DM>> { static constexpr bool value = true; };

// where the reverse passes find the dense arrays: M, H, invd (forward workspace) and Lc, invdc (factor
// of Hc) in LDS (WS / WSA), or in the tape slot in global memory (lean replay)
template <class P> struct AdjMats {
  P M, H, invd, Lc, invdc;
  GLBA float* Mb;  // lean unrolled replay: M-bar rows in the env's global scratch (else unused)
};

// per-env global scratch of the adjoint (after the env's row slab): per row (alpha, gamma, posbar),
// per contact kConAdjW floats: pos 3, frame 9, dist 1, geom1 (pos, axis) 6, geom2 (pos, axis) 6
constexpr int kConAdjW = 25;
__host__ __device__ inline int adj_scratch_floats(int nefc_max, int ncon_max) { return 3 * nefc_max + kConAdjW * ncon_max; }

// ------------------------------------------------------------------- unrolled mode: the solve tape
// Per env, in the unrolled scratch (capi.hip launch_vjp): the tape, then per-row accumulators.
//   header [4]: number of updates, of line searches, warm-start choice (0 qacc_warmstart, 1 smooth)
//   update k (k < KU): q_k [LD], grad_k [LD], Mgrad_k [LD], beta_k, num_k, den_k, -, active mask [2 NW]
//   line search k (k < KL): s_k [LD], alpha_k, nsets, -, -, weights [64], N [64], Q2 [64],
//     parent active masks [64][2 NW]: the accepted alpha_k = sum_j w_j N_j, where N_j = -Q1_j / Q2_j
//     is the Newton point of a point whose active set was A_j (tests/unrolled_solver_ref.py)
//   rows: arefb, Db, ca, cb [nefc_max] each, Jbar [nefc_max][LD]
struct TapeDims {
  int LD, NW, KU, KL, US, LSS, tape, stride;
  __host__ __device__ void init(int ld, int nefc_max, int iterations) {
    LD = ld;
    NW = (nefc_max + 63) / 64;
    if (NW < 1) NW = 1;
    const int it = iterations > 1 ? iterations : 1;
    KU = it + 1;
    KL = it;
    US = 3 * LD + 4 + 2 * NW;
    LSS = LD + 4 + 3 * 64 + 64 * 2 * NW;
    tape = 4 + KU * US + KL * LSS;
    stride = (tape + 4 * nefc_max + nefc_max * LD + 3) & ~3;
  }
};

struct SolveTape {
  static constexpr bool on = true;
  GLBA float* t;
  GLBA float* acc;  // the reverse sweep's row accumulators (t + d.tape, or the env's own scratch)
  TapeDims d;
  int nup, nls, nsets, overflow;
  INL GLBA float* upd(int k) const { return t + 4 + k * d.US; }
  INL GLBA float* ls(int k) const { return t + 4 + d.KU * d.US + k * d.LSS; }
  INL void put_mask(GLBA float* dst, int w, unsigned long long b, int lane) const {
    if (lane == 0) { dst[2 * w] = __uint_as_float((uint32_t)b); dst[2 * w + 1] = __uint_as_float((uint32_t)(b >> 32)); }
  }
  INL void warm(int wsel, int lane) {
    if (lane == 0) t[2] = (float)wsel;
  }
  template <class DD, bool G> INL void update(LDSA WS<DD>* W, Rows<G> R, int lane) {
    if (nup >= d.KU) { overflow = 1; return; }
    GLBA float* u = upd(nup);
    if (lane < d.LD) { u[lane] = W->qacc[lane]; u[d.LD + lane] = W->grad[lane]; u[2 * d.LD + lane] = 0.f; }
    for (int w = 0; w < d.NW; w++) {
      const int r = lane + 64 * w;
      put_mask(u + 3 * d.LD + 4, w, __ballot(r < W->nefc && R.jar[r] < 0.f), lane);
    }
    if (lane == 0) { u[3 * d.LD] = 0.f; u[3 * d.LD + 1] = 0.f; u[3 * d.LD + 2] = 0.f; }
    nup++;
  }
  INL void direction(float mg, float beta, float num, float den, int lane) {
    if (nup < 1 || overflow) return;
    GLBA float* u = upd(nup - 1);
    if (lane < d.LD) u[2 * d.LD + lane] = mg;
    if (lane == 0) { u[3 * d.LD] = beta; u[3 * d.LD + 1] = num; u[3 * d.LD + 2] = den; }
  }
  template <class DD> INL void ls_begin(LDSA WS<DD>* W, int lane) {
    nsets = 0;
    if (nls >= d.KL) { overflow = 1; return; }
    if (lane < d.LD) ls(nls)[lane] = W->search[lane];
  }
  // record the Newton point a_new of a point at a_par with f'' = d1 (its active set from the rows'
  // register / scratch copies exactly as the search's `partial` evaluates it); returns its index
  template <bool G> INL int add_set(Rows<G> R, int nefc, float a_par, float d1, float a_new, float ja0, float jv0,
                                    float ja1, float jv1, int lane) {
    const int idx = nsets < 64 ? nsets : 63;
    if (nsets >= 64) overflow = 1;
    nsets = nsets < 64 ? nsets + 1 : 64;
    if (nls >= d.KL) return idx;
    GLBA float* l = ls(nls);
    if (lane == 0) { l[d.LD + 4 + 64 + idx] = a_new; l[d.LD + 4 + 128 + idx] = d1; }
    GLBA float* mk = l + d.LD + 4 + 192 + idx * 2 * d.NW;
    put_mask(mk, 0, __ballot(ja0 + a_par * jv0 < 0.f), lane);
    if (d.NW > 1) put_mask(mk, 1, __ballot(ja1 + a_par * jv1 < 0.f), lane);
    for (int w = 2; w < d.NW; w++) {
      const int r = lane + 64 * w;
      put_mask(mk, w, __ballot(r < nefc && R.jar[r] + a_par * R.Jv[r] < 0.f), lane);
    }
    return idx;
  }
  INL void ls_end(float alpha, float rec, int lane) {
    if (nls >= d.KL) return;
    GLBA float* l = ls(nls);
    if (lane == 0) { l[d.LD] = alpha; l[d.LD + 1] = (float)nsets; }
    l[d.LD + 4 + lane] = rec;
    nls++;
  }
  INL void finish(int lane) {
    if (lane == 0) { t[0] = (float)nup; t[1] = (float)nls; t[3] = (float)overflow; }
  }
};

// wave sum of a 3-vector contribution into LDS dst (lane 0 writes)
INL void wsum3_into(LDSA float* dst, const float* v, int lane) {
  float a = wsum(v[0]), b = wsum(v[1]), c = wsum(v[2]);
  if (lane == 0) { dst[0] += a; dst[1] += b; dst[2] += c; }
}
// per-root reduction of lane-held subtree-com cotangents (only roots' scom are read forward)
template <class D, class AT> INL void scom_reduce(MP m, LDSA AT* A, int root_of_lane, const float* v, int lane) {
  for (int q = 0; q < m->nroot; q++) {
    const int r = m->root[q];
    float t[3] = {0.f, 0.f, 0.f};
    if (root_of_lane == r) { t[0] = v[0]; t[1] = v[1]; t[2] = v[2]; }
    wsum3_into(A->scomb[r], t, lane);
  }
}

// ------------------------------------------------------------------- env step (envs.py:333-492)
// Reward, aux' cotangents -> xpos / xquat of pelvis and head, qfrc_actuator, post-step qvel (in
// A->vtmp), input aux. Mirrors env_post branch for branch.
template <class D, class WT, class AT> INL void adj_env(MP m, LDSA WT* W, LDSA AT* A, CP c, const float* aux, float rb,
                                    const float* auxb_o, int lane) {
  const float dt = m->timestep;
  const float nj = (float)(m->nv - 6);
  if (lane >= 6 && lane < m->nv) {  // energy = ec mean|f v| + sc mean f^2 (reward has -energy)
    const float f = W->frc_act[lane], v = W->qvel[lane], sg = (f * v < 0.f) ? -1.f : 1.f;
    A->frcactb[lane] += -rb * (c->electricity_cost / nj * sg * v + c->stall_torque_cost / nj * 2.f * f);
    A->vtmp[lane] += -rb * c->electricity_cost / nj * sg * f;
  }
  if (lane == 0) {
    LDSA float* hp = W->xpos[c->head_body_id];
    LDSA float* bp = W->xpos[c->pelvis_body_id];
    LDSA float* bpb = A->xposb[c->pelvis_body_id];
    LDSA float* hpb = A->xposb[c->head_body_id];
    float tx = aux[1], ty = aux[2];
    const float db = xydist(tx, ty, bp), dh = xydist(tx, ty, hp);
    const float dist = fmaxf(db, dh);
    const bool close = dist < c->target_threshold;
    const float cc = close ? aux[4] + 1.f : 0.f;
    const bool adv = cc >= (float)c->stop_frames;
    const float tx2 = adv ? bp[0] + c->target_dist : tx, ty2 = adv ? bp[1] : ty;
    const float time = W->sc[SC_TIME];
    const float new_st = stance_of(c, W->sens);
    const bool changed = new_st != aux[5];
    (void)time;
    // aux' = {flip, tx2, ty2, tz2, cc', st', st_time', -dist2/dt, ep}
    A->auxb[0] += auxb_o[0];
    if (adv) { bpb[0] += auxb_o[1]; bpb[1] += auxb_o[2]; bpb[2] += auxb_o[3]; }
    else { A->auxb[1] += auxb_o[1]; A->auxb[2] += auxb_o[2]; A->auxb[3] += auxb_o[3]; }
    if (close && !adv) A->auxb[4] += auxb_o[4];
    if (!changed) { A->auxb[5] += auxb_o[5]; A->auxb[6] += auxb_o[6]; }
    A->auxb[8] += auxb_o[8];
    // d(dist2) from aux'[7] = -dist2 / dt
    float d2b = -auxb_o[7] / dt;
    {
      const float e_b = xydist(tx2, ty2, bp), e_h = xydist(tx2, ty2, hp);
      const bool pel = e_b >= e_h;
      LDSA float* p = pel ? bp : hp;
      LDSA float* pb = pel ? bpb : hpb;
      const float e = pel ? e_b : e_h;
      if (e > 0.f) {
        const float gx = d2b * (p[0] - tx2) / e, gy = d2b * (p[1] - ty2) / e;
        pb[0] += gx; pb[1] += gy;
        if (adv) { bpb[0] -= gx; bpb[1] -= gy; }  // tx2 = bp[0] + const, ty2 = bp[1]
        else { A->auxb[1] -= gx; A->auxb[2] -= gy; }
      }
    }
    // progress = (-dist/dt - aux[7]) * w
    const float w = c->progress_weight;
    A->auxb[7] += -w * rb;
    const float distb = -w / dt * rb;
    {
      const bool pel = db >= dh;
      LDSA float* p = pel ? bp : hp;
      LDSA float* pb = pel ? bpb : hpb;
      const float e = pel ? db : dh;
      if (e > 0.f) {
        const float gx = distb * (p[0] - tx) / e, gy = distb * (p[1] - ty) / e;
        pb[0] += gx; pb[1] += gy;
        A->auxb[1] -= gx; A->auxb[2] -= gy;
      }
    }
    // posture = wp (|pitch| outside (-0.087, 0.174) + |roll| outside (-0.174, 0.174))
    if (c->posture_penalty_weight != 0.f) {
      LDSA float* q = W->xquat[c->pelvis_body_id];
      LDSA float* qb = A->xquatb[c->pelvis_body_id];
      const float qw = q[0], qx = q[1], qy = q[2], qz = q[3];
      float roll, pitch, yaw;
      rpy(q, roll, pitch, yaw);
      const float wp = -rb * c->posture_penalty_weight;
      const float pitchb = ((pitch > -0.087f) && (pitch < 0.174f)) ? 0.f : wp * (pitch < 0.f ? -1.f : 1.f);
      const float rollb = ((roll > -0.174f) && (roll < 0.174f)) ? 0.f : wp * (roll < 0.f ? -1.f : 1.f);
      const float sp = 2.f * (qw * qy - qz * qx);
      if (sp > -1.f && sp < 1.f) {
        const float spb = pitchb / sqrtf(1.f - sp * sp);
        qb[0] += 2.f * qy * spb; qb[2] += 2.f * qw * spb; qb[3] -= 2.f * qx * spb; qb[1] -= 2.f * qz * spb;
      }
      const float ra = 2.f * (qw * qx + qy * qz), rbb = 1.f - 2.f * (qx * qx + qy * qy), den = ra * ra + rbb * rbb;
      if (den > 0.f) {
        const float ab = rollb * rbb / den, bb = -rollb * ra / den;
        qb[0] += 2.f * qx * ab; qb[1] += 2.f * qw * ab; qb[2] += 2.f * qz * ab; qb[3] += 2.f * qy * ab;
        qb[1] += -4.f * qx * bb; qb[2] += -4.f * qy * bb;
      }
    }
  }
  SYNC();
}

// ------------------------------------------------------------------- integration (forward.py)
// in: A->vtmp = cotangent of qvel', gq = cotangent of qpos' (global). out: A->qposb, A->qvelb,
// A->qaccb, A->Mb (implicit / eulerdamp matrix path); unrolled mode: the matrix path's force is
// qfrc_smooth + qfrc_constraint (A->frcsb, A->qfcb), not M qacc.
template <class D, class WT, class AT, class MT> INL void adj_integrate(MP m, LDSA WT* W, LDSA AT* A, const MT& mt,
                                                                      const float* gq, bool unr, int lane) {
  constexpr int LD = D::LD;
  const int nv = m->nv;
  const float dt = m->timestep;
  // lean replay: the implicit-integration factor's row and column come from the slot in global
  // memory; their loads go out before the joint pass, whose work hides their latency
  [[maybe_unused]] CholOps<D::NV> hops;
  if constexpr (is_lean<AT>::value) hops = chol_load<D>(mt.H, mt.invd, lane);
  if (lane < m->njnt) {
    const JntRec jr = ldrec(&m->jrec[lane]);
    const int q = jr.qadr, d = jr.dofadr;
    if (jr.isfree) {
      for (int i = 0; i < 3; i++) { A->qposb[q + i] += gq[q + i]; A->vtmp[d + i] += dt * gq[q + i]; }
      // quat' = normalize(q0 (x) qr), qr = (cos th, w^ sin th), th = |w| dt / 2, w = qvel'[3:6]
      float w[3] = {W->qvel[d + 3], W->qvel[d + 4], W->qvel[d + 5]};
      float wn[3] = {w[0], w[1], w[2]};
      const float nrm = norm3(wn);
      float s, cth;
      sincosf(0.5f * nrm * dt, &s, &cth);
      const float qr[4] = {cth, wn[0] * s, wn[1] * s, wn[2] * s};
      const float q0[4] = {A->qpos0[q + 3], A->qpos0[q + 4], A->qpos0[q + 5], A->qpos0[q + 6]};
      float pq[4];
      qmul(pq, q0, qr);
      const float qb[4] = {gq[q + 3], gq[q + 4], gq[q + 5], gq[q + 6]};
      float pb[4] = {0.f, 0.f, 0.f, 0.f}, q0b[4] = {0.f, 0.f, 0.f, 0.f}, qrb[4] = {0.f, 0.f, 0.f, 0.f};
      qnorm_adj(pq, qb, pb);
      qmul_adj(q0, qr, pb, q0b, qrb);
      for (int i = 0; i < 4; i++) A->qposb[q + 3 + i] += q0b[i];
      const float thb = -s * qrb[0] + cth * (wn[0] * qrb[1] + wn[1] * qrb[2] + wn[2] * qrb[3]);
      const float wnb[3] = {s * qrb[1], s * qrb[2], s * qrb[3]};
      float wb[3] = {0.f, 0.f, 0.f};
      norm3_adj(w, wnb, wb);
      if (nrm > 0.f) { const float nb = 0.5f * dt * thb / nrm; wb[0] += nb * w[0]; wb[1] += nb * w[1]; wb[2] += nb * w[2]; }
      for (int i = 0; i < 3; i++) A->vtmp[d + 3 + i] += wb[i];
    } else {
      A->qposb[q] += gq[q];
      A->vtmp[d] += dt * gq[q];
    }
  }
  SYNC();
  // qvel' = qvel + dt a'
  float apb = 0.f;
  if (lane < nv) { A->qvelb[lane] += A->vtmp[lane]; apb = dt * A->vtmp[lane]; }
  const bool damp = (m->integrator == MJL_INT_IMPLICITFAST || m->eulerdamp) && m->any_damping;
  if (damp) {  // a' = Hd^-1 (M qacc), Hd = M + dt diag(damping), factor in W->H
    if (lane < LD) A->rb[lane] = (lane < nv) ? apb : 0.f;
    SYNC();
    const float rx = lane < nv ? A->rb[lane] : 0.f;
    float r;
    if constexpr (is_lean<AT>::value) r = chol_apply(hops, rx);
    else r = chol_solve<D>(mt.H, mt.invd, rx, lane);
    SYNC();
    if (lane < LD) A->rb[lane] = (lane < nv) ? r : 0.f;
    SYNC();
    if (lane < nv) {
      const float rl = A->rb[lane];
      if (unr) {  // a' = Hd^-1 (qfrc_smooth + qfrc_constraint)
        if constexpr (is_lean<AT>::value) {
          GLBA float* row = mt.Mb + lane * LD;  // zeroed at kernel start
          for (int k = 0; k < nv; k++) row[k] -= rl * A->ap[k];
        } else {
          for (int k = 0; k < nv; k++) A->Mb[lane * LD + k] -= rl * A->ap[k];
        }
        A->frcsb[lane] += rl;
        A->qfcb[lane] += rl;
      } else {
        // lean: M-bar's term rb (qacc - a')^T is formed in adj_mass
        if constexpr (!is_lean<AT>::value)
          for (int k = 0; k < nv; k++) A->Mb[lane * LD + k] += rl * (W->qacc[k] - A->ap[k]);
        A->qaccb[lane] += rowdot<LD>(mt.M + lane * LD, A->rb);  // (M rb)[lane] (mrow)
      }
    }
  } else if (lane < nv) {
    A->qaccb[lane] += apb;
  }
  SYNC();
}

// ------------------------------------------------------------------- constraint solve + rows
// Per row, from the cotangents of its aref and D: alpha (J-bar coefficient of qvel: aref = -b J qvel
// - k imp pos), gamma (J-bar coefficient of qacc, implicit mode), posbar -> global scratch; then
// qvel-bar += sum_r alpha_r J_r and the limit rows' pos -> qpos-bar.
template <class D> INL void adj_row_map(MP m, Rows<true> R, GLBA float* scr, int nefc_max, int r, float arefb,
                                        float Db, float gam) {
  GLBA float* alpha = scr;
  GLBA float* gamma = scr + nefc_max;
  GLBA float* posb = scr + 2 * nefc_max;
  const int meta = R.emeta[r], type = meta >> 16, id = meta & 0xffff;
  const CSTA float *sr, *si;
  if (type == 0) { sr = m->jnt_solref[id]; si = m->jnt_solimp[id]; }
  else if (type == 1) { sr = m->tendon_solref[id]; si = m->tendon_solimp[id]; }
  else { sr = m->pair_solref[id]; si = m->pair_solimp[id]; }
  float k, b, imp;
  const float pos = R.epos[r];
  kbi(m->timestep, sr, si, pos, k, b, imp);
  const float invw = R.einvw[r];
  const float rr = invw * (1.f - imp) / imp;
  const float dDdimp = (rr > kMinVal) ? 1.f / (invw * (1.f - imp) * (1.f - imp)) : 0.f;
  const float impb = -k * pos * arefb + Db * dDdimp;
  alpha[r] = -b * arefb;
  gamma[r] = gam;
  posb[r] = -k * imp * arefb + impb * imp_dpos(si, pos);
}

template <class D, class WT, class AT> INL void adj_rows_tail(MP m, LDSA WT* W, LDSA AT* A, Rows<true> R, GLBA float* scr,
                                          int nefc_max, int lane) {
  constexpr int LD = D::LD;
  const int nv = m->nv, nefc = W->nefc;
  GLBA float* alpha = scr;
  GLBA float* posb = scr + 2 * nefc_max;
  if (lane < nv) {  // qvel-bar += sum_r alpha_r J_r  (aref depends on J qvel)
    float s = 0.f;
    for (int r = 0; r < nefc; r++) s += alpha[r] * R.J[r * LD + lane];
    A->qvelb[lane] += s;
  }
  if (lane == 0) {  // limit rows: pos = min(q - lo, hi - q) - margin (serial: tendons may share joints)
    for (int r = 0; r < W->nlim; r++) {
      const int meta = R.emeta[r], type = meta >> 16, id = meta & 0xffff;
      const float pb = posb[r];
      if (type == 0) {
        const int qa = m->jnt_qposadr[id];
        const float q = A->qpos0[qa];
        const float sg = (q - m->jnt_range[id][0] < m->jnt_range[id][1] - q) ? 1.f : -1.f;
        A->qposb[qa] += sg * pb;
      } else {
        const float len = W->tenlen[id];
        const float sg = (len - m->tendon_range[id][0] < m->tendon_range[id][1] - len) ? 1.f : -1.f;
        for (int w = 0; w < m->tendon_num[id]; w++) A->qposb[m->tendon_qadr[id][w]] += sg * m->tendon_coef[id][w] * pb;
      }
    }
  }
  SYNC();
}

// Implicit mode: derivative at the converged active set (mu = Hc^-1 qacc-bar).
template <class D, class WT, class AT, class MT> INL void adj_solver_rows(MP m, LDSA WT* W, LDSA AT* A, const MT& mt,
                                                                        Rows<true> R, GLBA float* scr, int nefc_max,
                                                                        int lane) {
  constexpr int LD = D::LD;
  const int nv = m->nv, nefc = W->nefc;
  const float mu = chol_solve<D>(mt.Lc, mt.invdc, lane < nv ? A->qaccb[lane] : 0.f, lane);
  if (lane < LD) A->mu[lane] = (lane < nv) ? mu : 0.f;
  SYNC();
  if (lane < nv) {
    A->frcsb[lane] += A->mu[lane];
    if constexpr (!is_lean<AT>::value) {  // lean: M-bar's term -mu qacc^T formed in adj_mass
      const float ml = A->mu[lane];
      for (int k = 0; k < nv; k++) A->Mb[lane * LD + k] -= ml * W->qacc[k];
    }
  }
  for (int r = lane; r < nefc; r += 64) {
    const float jar = R.jar[r], Dr = R.D[r];
    const bool act = jar < 0.f;
    float jm = 0.f;
    for (int k = 0; k < LD; k++) jm += R.J[r * LD + k] * A->mu[k];
    adj_row_map<D>(m, R, scr, nefc_max, r, act ? Dr * jm : 0.f, act ? -jm * jar : 0.f, act ? -Dr * jm : 0.f);
  }
  SYNC();
  adj_rows_tail<D>(m, W, A, R, scr, nefc_max, lane);
}

// Unrolled mode: reverse sweep of the taped solve (tests/unrolled_solver_ref.py solve_vjp, line by
// line). In: A->qaccb, A->qfcb (cotangents of the final qacc and qfrc_constraint). Out: A->Mb,
// A->frcsb, the per-row aref / D cotangents (mapped by adj_row_map) and J-bar rows (u.rows Jbar,
// read by adj_contact_jac). Vectors are lane-resident (lane = dof); uv[] stages M v / J v operands.
// Lean replay (CG only): chol(M) comes from the tape slot (the record step's forward factor), and the
// lane's M-bar row accumulates in registers between one load and one store of its global scratch row.
template <class D, class WT, class AT, class MT>
INL void adj_solver_unrolled(MP m, LDSA WT* W, LDSA AT* A, const MT& mt, Rows<true> R, GLBA float* scr, int nefc_max,
                             const SolveTape& tp, int lane) {
  constexpr int LD = D::LD;
  constexpr bool LEAN = is_lean<AT>::value;
  const int nv = m->nv, nefc = W->nefc;
  const bool cg = m->solver != MJL_SOLVER_NEWTON;
  const TapeDims& d = tp.d;
  GLBA float* arefb = tp.acc;
  GLBA float* Dbar = arefb + nefc_max;
  GLBA float* ca = arefb + 2 * nefc_max;
  GLBA float* cb = arefb + 3 * nefc_max;
  GLBA float* Jbar = arefb + 4 * nefc_max;
  LDSA float* V1 = A->uv[0];
  LDSA float* V2 = A->uv[1];
  LDSA float* V3 = A->uv[2];
  const bool isd = lane < nv;
  auto ld = [&](auto p) -> float { return isd ? p[lane] : 0.f; };
  auto stage = [&](LDSA float* dst, float v) { if (lane < LD) dst[lane] = isd ? v : 0.f; };
  auto bit = [&](GLBA const float* mk, int r) -> bool {
    const uint32_t w = __float_as_uint(mk[2 * (r >> 6) + ((r >> 5) & 1)]);
    return (w >> (r & 31)) & 1u;
  };
  // J-bar rows += ca (x) va + cb (x) vb (ca, cb per row in scratch; va, vb in LDS); JB rows per step
  // with every load issued before the stores: each step is one global round trip (4 rows per step:
  // 32-row sweeps waited 8; single read-modify-writes waited for each one)
  constexpr int JB = 16;
  auto jbar_add = [&](LDSA const float* va, LDSA const float* vb) {
    SYNC();
    if (isd) {
      const float a = va[lane], b = vb[lane];
      int r = 0;
      for (; r + JB <= nefc; r += JB) {
        float c0[JB], c1[JB], jb[JB];
#pragma unroll
        for (int e = 0; e < JB; e++) { c0[e] = ca[r + e]; c1[e] = cb[r + e]; jb[e] = Jbar[(r + e) * LD + lane]; }
#pragma unroll
        for (int e = 0; e < JB; e++) Jbar[(r + e) * LD + lane] = jb[e] + (c0[e] * a + c1[e] * b);
      }
      for (; r + 4 <= nefc; r += 4) {
        float c0[4], c1[4], jb[4];
#pragma unroll
        for (int e = 0; e < 4; e++) { c0[e] = ca[r + e]; c1[e] = cb[r + e]; jb[e] = Jbar[(r + e) * LD + lane]; }
#pragma unroll
        for (int e = 0; e < 4; e++) Jbar[(r + e) * LD + lane] = jb[e] + (c0[e] * a + c1[e] * b);
      }
      for (; r < nefc; r++) Jbar[r * LD + lane] += ca[r] * a + cb[r] * b;
    }
  };
  auto jt = [&](GLBA const float* c) -> float {  // (J' c)[lane] in row order, JB rows' loads per step
    float x = 0.f;
    if (isd) {
      int r = 0;
      for (; r + JB <= nefc; r += JB) {
        float jv[JB], cv[JB];
#pragma unroll
        for (int e = 0; e < JB; e++) { jv[e] = R.J[(r + e) * LD + lane]; cv[e] = c[r + e]; }
#pragma unroll
        for (int e = 0; e < JB; e++) x += jv[e] * cv[e];
      }
      for (; r + 4 <= nefc; r += 4) {
        float jv[4], cv[4];
#pragma unroll
        for (int e = 0; e < 4; e++) { jv[e] = R.J[(r + e) * LD + lane]; cv[e] = c[r + e]; }
#pragma unroll
        for (int e = 0; e < 4; e++) x += jv[e] * cv[e];
      }
      for (; r < nefc; r++) x += R.J[r * LD + lane] * c[r];
    }
    return x;
  };
  float mbr[LEAN ? LD : 1];  // lean: this lane's M-bar row
  if constexpr (LEAN) {
    const GLBA f32x4* g = (const GLBA f32x4*)(mt.Mb + (isd ? lane : 0) * LD);
#pragma unroll
    for (int q = 0; q < LD / 4; q++) {
      const f32x4 x = g[q];
#pragma unroll
      for (int e = 0; e < 4; e++) mbr[4 * q + e] = x[e];
    }
  }
  auto mb_outer = [&](float a, LDSA const float* v) {  // Mb[lane][:] += a v' (v zero beyond nv)
    if (isd) {
      const LDSA f32x4* vv = (const LDSA f32x4*)v;
      if constexpr (LEAN) {
#pragma unroll
        for (int q = 0; q < LD / 4; q++) {
          const f32x4 y = vv[q];
#pragma unroll
          for (int e = 0; e < 4; e++) mbr[4 * q + e] += a * y[e];
        }
      } else {
        LDSA f32x4* row = (LDSA f32x4*)(A->Mb + lane * LD);
#pragma unroll
        for (int q = 0; q < LD / 4; q++) {
          f32x4 x = row[q];
          const f32x4 y = vv[q];
#pragma unroll
          for (int e = 0; e < 4; e++) x[e] += a * y[e];
          row[q] = x;
        }
      }
    }
  };
  for (int r = lane; r < nefc; r += 64) { arefb[r] = 0.f; Dbar[r] = 0.f; }
  if (isd)
    for (int r = 0; r < nefc; r++) Jbar[r * LD + lane] = 0.f;
  const int nup = (int)tp.t[0], nls = (int)tp.t[1], K = nup - 1;
  const int wsel = nup > 0 ? (int)tp.t[2] : 1;
  // L(M) in A->Lc (CG preconditioner; the smooth warm start); lean: mt.Lc, the slot's copy
  if constexpr (!LEAN) {
    stage(V1, 0.f);
    SYNC();
    chol_factor_solve<D>(W->M, A->Lc, A->invdc, nv, V1, lane);
    SYNC();
  }
  float qb = ld(A->qaccb), sb = 0.f, gb = 0.f, mgb = 0.f;
  for (int k = K; k >= 0; k--) {
    GLBA const float* u = tp.upd(k);
    const float q_k = ld(u), grad_k = ld(u + LD), mg_k = ld(u + 2 * LD);
    float sbp = 0.f, gbp = 0.f, mgbp = 0.f;
    if (k < nls) {  // s_k = -Mg_k + beta_k s_{k-1} was used by line search k
      mgb -= sb;
      if (cg && k >= 1) {
        GLBA const float* up = tp.upd(k - 1);
        const float betab = wsum(sb * ld(tp.ls(k - 1)));
        const float beta = u[3 * LD], num = u[3 * LD + 1], den_raw = u[3 * LD + 2];
        sbp += beta * sb;
        const float den = fmaxf(kMinVal, den_raw);
        if (num / den > 0.f) {
          const float nb = betab / den;
          gb += nb * (mg_k - ld(up + 2 * LD));
          mgb += nb * grad_k;
          mgbp -= nb * grad_k;
          if (den_raw > kMinVal) {
            const float denb = -betab * num / (den * den);
            gbp += denb * ld(up + 2 * LD);
            mgbp += denb * ld(up + LD);
          }
        }
      }
    }
    // Mg_k = P_k^-1 grad_k
    if (__ballot(isd && mgb != 0.f) != 0ull) {
      float lam;
      stage(V1, mgb);
      stage(V2, mg_k);
      SYNC();
      if (LEAN || cg) {
        lam = chol_solve<D>(mt.Lc, mt.invdc, mgb, lane);
      } else if constexpr (!LEAN) {  // H_k = M + J' D_A J over update k's active rows (the tape's mask)
        for (int r = lane; r < nefc; r += 64) R.jar[r] = bit(u + 3 * LD + 4, r) ? -1.f : 1.f;
        SYNC();
        if constexpr (D::NV < 32) {
          const f32x16 acc = solver_hessian_acc<D, true>(m, W, R, lane);
          lam = chol_aug_factor_solve<D, true>(W->M, A->Lc, A->invdc, nv, V1, lane, acc);
        } else {
          solver_hessian<D, true>(m, W, R, lane);
          lam = chol_factor_solve<D>(W->H, W->H, W->invd, nv, V1, lane);
        }
        SYNC();
        stage(V3, lam);
        SYNC();
        for (int r = lane; r < nefc; r += 64) {
          const bool act = bit(u + 3 * LD + 4, r);
          const float Jl = rowdot<LD>(R.J + r * LD, V3), Jm = rowdot<LD>(R.J + r * LD, V2), Dr = R.D[r];
          if (act) Dbar[r] -= Jl * Jm;
          ca[r] = act ? -Dr * Jm : 0.f;
          cb[r] = act ? -Dr * Jl : 0.f;
        }
        jbar_add(V3, V2);
      }
      if (!isd) lam = 0.f;
      mb_outer(-lam, V2);
      gb += lam;
      SYNC();
    }
    // grad_k = M q_k - f - J' force_k  (+ the final qfrc_constraint's cotangent at k = K)
    const float qfcb = -gb + (k == K ? ld(A->qfcb) : 0.f);
    if (isd) A->frcsb[lane] -= gb;
    stage(V1, gb);
    stage(V2, q_k);
    stage(V3, qfcb);
    SYNC();
    qb += isd ? rowdot<LD>(mt.M + lane * LD, V1) : 0.f;  // (M gb)[lane]
    mb_outer(gb, V2);
    for (int r = lane; r < nefc; r += 64) {
      const bool act = bit(u + 3 * LD + 4, r);
      const float jar = rowdot<LD>(R.J + r * LD, V2) - R.aref[r], Dr = R.D[r];
      const float force = act ? -Dr * jar : 0.f;
      const float forceb = rowdot<LD>(R.J + r * LD, V3);
      ca[r] = force;
      cb[r] = act ? -forceb * Dr : 0.f;  // jar-bar
      if (act) { Dbar[r] -= forceb * jar; arefb[r] += forceb * Dr; }
    }
    jbar_add(V3, V2);
    SYNC();
    qb += jt(cb);
    if (k == 0) break;
    // line search k-1 and q_k = q_{k-1} + alpha s_{k-1}
    GLBA const float* l = tp.ls(k - 1);
    GLBA const float* up = tp.upd(k - 1);
    const float s = ld(l), qp = ld(up), alpha = l[LD];
    const int ns = (int)l[LD + 1];
    const float alphab = wsum(qb * s);
    sbp += alpha * qb;
    float q1b = 0.f, q2b = 0.f;
    if (lane < ns) {
      const float w = l[LD + 4 + lane], N = l[LD + 4 + 64 + lane], Q2 = l[LD + 4 + 128 + lane];
      if (w != 0.f) { q1b = alphab * w * (-1.f / Q2); q2b = alphab * w * (-N / Q2); }
    }
    const float c1b = wsum(q1b), c2b = wsum(q2b);
    stage(V1, s);
    stage(V2, qp);
    SYNC();
    for (int r = lane; r < nefc; r += 64) {
      float ra = 0.f, rb = 0.f;
      for (int j = 0; j < ns; j++) {
        const float a = rdlane(q1b, j), b = rdlane(q2b, j);
        if (bit(l + LD + 4 + 192 + j * 2 * d.NW, r)) { ra += a; rb += b; }
      }
      const float jar = rowdot<LD>(R.J + r * LD, V2) - R.aref[r], Jv = rowdot<LD>(R.J + r * LD, V1), Dr = R.D[r];
      Dbar[r] += ra * Jv * jar + rb * Jv * Jv;
      ca[r] = ra * Dr * jar + 2.f * rb * Dr * Jv;  // Jv-bar
      cb[r] = ra * Dr * Jv;                        // jar-bar
      arefb[r] -= ra * Dr * Jv;
    }
    jbar_add(V1, V2);
    SYNC();
    const float Ms = isd ? rowdot<LD>(mt.M + lane * LD, V1) : 0.f, Mq = isd ? rowdot<LD>(mt.M + lane * LD, V2) : 0.f;
    const float f = ld(W->frc_smooth);
    sbp += c1b * (Mq - f) + 2.f * c2b * Ms + jt(ca);
    qb += c1b * Ms + jt(cb);
    mb_outer(c1b * s, V2);
    mb_outer(c2b * s, V1);
    if (isd) A->frcsb[lane] -= c1b * s;
    sb = sbp;
    gb = gbp;
    mgb = mgbp;
    SYNC();
  }
  if (wsel == 1) {  // q_0 = qacc_smooth = M^-1 f (Newton's Hessians overwrote A->Lc: refactor M)
    stage(V1, qb);
    SYNC();
    float lam;
    if constexpr (LEAN) lam = chol_solve<D>(mt.Lc, mt.invdc, qb, lane);
    else if (cg) lam = chol_solve<D>(mt.Lc, mt.invdc, qb, lane);
    else lam = chol_factor_solve<D>(W->M, A->Lc, A->invdc, nv, V1, lane);
    if (!isd) lam = 0.f;
    if (isd) A->frcsb[lane] += lam;
    mb_outer(-lam, W->qacc_smooth);
  } else if (isd) {  // q_0 = qacc_warmstart: jax.grad carries this cotangent to the previous step
    A->wsb[lane] = qb;
  }
  if constexpr (LEAN) {  // the M-bar row back to its scratch row (adj_mass reads it)
    if (isd) {
      GLBA f32x4* g = (GLBA f32x4*)(mt.Mb + lane * LD);
#pragma unroll
      for (int q = 0; q < LD / 4; q++) {
        f32x4 x;
#pragma unroll
        for (int e = 0; e < 4; e++) x[e] = mbr[4 * q + e];
        g[q] = x;
      }
    }
  }
  SYNC();
  for (int r = lane; r < nefc; r += 64) adj_row_map<D>(m, R, scr, nefc_max, r, arefb[r], Dbar[r], 0.f);
  SYNC();
  adj_rows_tail<D>(m, W, A, R, scr, nefc_max, lane);
}

// ------------------------------------------------------------------- contact Jacobians
// J rows of contact c from Jp_d = s_d (cdof_lin_d + cdof_ang_d x (pos - scom_root)); lanes 0..31 =
// dof. Accumulates cdof-bar (lane-owned), scom-bar (per root), and the contact's pos / frame /
// dist cotangents into the scratch record.
template <class D, class WT, class AT> INL void adj_contact_jac(MP m, LDSA WT* W, LDSA AT* A, Rows<true> R, GLBA float* scr,
                                            int nefc_max, GLBA const float* Jbar, int lane) {
  constexpr int LD = D::LD;
  const int nv = m->nv, ncon = W->ncon;
  GLBA float* alpha = scr;
  GLBA float* gamma = scr + nefc_max;
  GLBA float* posb = scr + 2 * nefc_max;
  GLBA float* conb = scr + 3 * nefc_max;
  const int d = lane;
  const bool isd = lane < nv;
  const int root = isd ? ldrec(&m->drec[d]).rootid : 0;
  float scb[3] = {0.f, 0.f, 0.f};
  for (int c = 0; c < ncon; c++) {
    GLBA float* cr = R.con + c * CONW;
    const int packed = __float_as_int(cr[15]), dim = (packed >> 16) & 0xff;
    const uint32_t mask1 = __float_as_uint(cr[12]), mask2 = __float_as_uint(cr[13]);
    const float muf = cr[14];
    const int r0 = R.con_efc[c], nrow = dim == 1 ? 1 : 4;
    float jn = 0.f, jt1 = 0.f, jt2 = 0.f, pb = 0.f;
    if (isd) {
      const float qv = A->qvel0[d], mu = A->mu[d], qa = W->qacc[d];
      float Jb[4];
      for (int q = 0; q < nrow; q++) {
        const int r = r0 + q;
        Jb[q] = alpha[r] * qv + R.force[r] * mu + gamma[r] * qa;
        if (Jbar) Jb[q] += Jbar[r * D::LD + d];  // unrolled mode: the full J-bar rows
      }
      if (dim == 1) jn = Jb[0];
      else { jn = Jb[0] + Jb[1] + Jb[2] + Jb[3]; jt1 = muf * (Jb[0] - Jb[1]); jt2 = muf * (Jb[2] - Jb[3]); }
    }
    if (lane < nrow) pb = posb[r0 + lane];
    const float distb = wsum(pb);
    float nb[3] = {0.f, 0.f, 0.f}, t1b[3] = {0.f, 0.f, 0.f}, t2b[3] = {0.f, 0.f, 0.f}, offb[3] = {0.f, 0.f, 0.f};
    const float s = isd ? (float)((mask2 >> d) & 1u) - (float)((mask1 >> d) & 1u) : 0.f;
    if (s != 0.f) {
      const float cd[6] = {W->cdof[d][0], W->cdof[d][1], W->cdof[d][2], W->cdof[d][3], W->cdof[d][4], W->cdof[d][5]};
      const float off[3] = {cr[0] - W->scom[root][0], cr[1] - W->scom[root][1], cr[2] - W->scom[root][2]};
      float cx[3];
      cross3(cx, cd, off);
      const float jp[3] = {s * (cd[3] + cx[0]), s * (cd[4] + cx[1]), s * (cd[5] + cx[2])};
      for (int i = 0; i < 3; i++) { nb[i] = jn * jp[i]; t1b[i] = jt1 * jp[i]; t2b[i] = jt2 * jp[i]; }
      float jpb[3];
      for (int i = 0; i < 3; i++) jpb[i] = jn * cr[3 + i] + jt1 * cr[6 + i] + jt2 * cr[9 + i];
      // jp = s (lin + ang x off)
      for (int i = 0; i < 3; i++) A->cdofb[d][3 + i] += s * jpb[i];
      const float sjpb[3] = {s * jpb[0], s * jpb[1], s * jpb[2]};
      float angb[3] = {0.f, 0.f, 0.f};
      cross3_adj(cd, off, sjpb, angb, offb);
      for (int i = 0; i < 3; i++) { A->cdofb[d][i] += angb[i]; scb[i] -= offb[i]; }
    }
    float v[13];
    for (int i = 0; i < 3; i++) { v[i] = wsum(offb[i]); v[3 + i] = wsum(nb[i]); v[6 + i] = wsum(t1b[i]); v[9 + i] = wsum(t2b[i]); }
    v[12] = distb;
    if (lane < 13) conb[c * kConAdjW + lane] = v[lane];
  }
  scom_reduce<D>(m, A, isd ? root : -1, scb, lane);
  SYNC();
}

// ------------------------------------------------------------------- collision (collide())
// frame rows: n, t1, t2. In: dist / pos / frame cotangents; out: cotangents of the geoms' centre
// and z axis. Each branch recomputes the forward's intermediate values with the same operations.
INL void make_frame_adj(const float* a_in, const float* fb, float* a_inb) {
  float a[3] = {a_in[0], a_in[1], a_in[2]};
  norm3(a);
  float b0[3] = {0.f, 0.f, 0.f};
  if (a[1] > -0.5f && a[1] < 0.5f) b0[1] = 1.f; else b0[2] = 1.f;
  const float ab = dot3(a, b0);
  float braw[3] = {b0[0] - a[0] * ab, b0[1] - a[1] * ab, b0[2] - a[2] * ab};
  float b[3] = {braw[0], braw[1], braw[2]};
  norm3(b);
  float abar[3] = {fb[0], fb[1], fb[2]}, bbar[3] = {fb[3], fb[4], fb[5]};
  cross3_adj(a, b, fb + 6, abar, bbar);
  float brawb[3] = {0.f, 0.f, 0.f};
  norm3_adj(braw, bbar, brawb);
  const float abb = -dot3(a, brawb);
  for (int i = 0; i < 3; i++) abar[i] += -ab * brawb[i] + abb * b0[i];
  norm3_adj(a_in, abar, a_inb);
}
// seg_point(r, a, b, pt) adjoint
INL void seg_point_adj(const float* a, const float* b, const float* pt, const float* rb, float* ab_, float* bb_,
                       float* ptb) {
  const float ab[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
  const float ap[3] = {pt[0] - a[0], pt[1] - a[1], pt[2] - a[2]};
  const float num = dot3(ap, ab), den = dot3(ab, ab) + 1e-6f;
  const float t0 = num / den, t = fminf(fmaxf(t0, 0.f), 1.f);
  float abb[3] = {t * rb[0], t * rb[1], t * rb[2]};
  for (int i = 0; i < 3; i++) ab_[i] += rb[i];
  const float tb = dot3(rb, ab);
  if (t0 > 0.f && t0 < 1.f) {
    const float numb = tb / den, denb = -tb * num / (den * den);
    for (int i = 0; i < 3; i++) {
      const float apb = numb * ab[i];
      abb[i] += numb * ap[i] + 2.f * denb * ab[i];
      ptb[i] += apb; ab_[i] -= apb;
    }
  }
  for (int i = 0; i < 3; i++) { bb_[i] += abb[i]; ab_[i] -= abb[i]; }
}
template <class D, class WT> INL void collide_adj(const PairRec& pr, LDSA WT* W, int k, float distb, const float* posb,
                                        const float* frb, float* x1b, float* z1b, float* x2b, float* z2b) {
  const int kind = pr.kind, g1 = pr.g1, g2 = pr.g2;
  const float x1[3] = {W->gpos[g1][0], W->gpos[g1][1], W->gpos[g1][2]};
  const float x2[3] = {W->gpos[g2][0], W->gpos[g2][1], W->gpos[g2][2]};
  const float z1[3] = {W->gaxis[g1][0], W->gaxis[g1][1], W->gaxis[g1][2]};
  const float z2[3] = {W->gaxis[g2][0], W->gaxis[g2][1], W->gaxis[g2][2]};
  const float r1 = pr.r1, r2 = pr.r2, h1 = pr.h1, h2 = pr.h2;
  if (kind == MJL_COL_PLANE_SPHERE) {
    const float d[3] = {x2[0] - x1[0], x2[1] - x1[1], x2[2] - x1[2]};
    const float dist = dot3(d, z1) - r2, s = r2 + 0.5f * dist;
    for (int i = 0; i < 3; i++) { x2b[i] += posb[i]; z1b[i] -= s * posb[i]; }
    distb += 0.5f * -dot3(z1, posb);
    for (int i = 0; i < 3; i++) { z1b[i] += distb * d[i]; x2b[i] += distb * z1[i]; x1b[i] -= distb * z1[i]; }
    make_frame_adj(z1, frb, z1b);
    return;
  }
  if (kind == MJL_COL_PLANE_CAPSULE) {
    const float* n = z1;
    const float nd = dot3(n, z2);
    const float braw[3] = {z2[0] - n[0] * nd, z2[1] - n[1] * nd, z2[2] - n[2] * nd};
    float b[3] = {braw[0], braw[1], braw[2]};
    const float bn = norm3(b);
    if (bn < 0.5f) { b[0] = 0.f; b[1] = 0.f; b[2] = 0.f; if (n[1] > -0.5f && n[1] < 0.5f) b[1] = 1.f; else b[2] = 1.f; }
    const float sg = (k == 0) ? 1.f : -1.f;
    const float sp[3] = {x2[0] + sg * z2[0] * h2, x2[1] + sg * z2[1] * h2, x2[2] + sg * z2[2] * h2};
    const float d[3] = {sp[0] - x1[0], sp[1] - x1[1], sp[2] - x1[2]};
    const float dist = dot3(d, n) - r2, s = r2 + 0.5f * dist;
    float nb[3] = {frb[0], frb[1], frb[2]}, bb[3] = {frb[3], frb[4], frb[5]}, spb[3];
    for (int i = 0; i < 3; i++) { spb[i] = posb[i]; nb[i] -= s * posb[i]; }
    distb += 0.5f * -dot3(n, posb);
    for (int i = 0; i < 3; i++) { spb[i] += distb * n[i]; x1b[i] -= distb * n[i]; nb[i] += distb * d[i]; }
    cross3_adj(n, b, frb + 6, nb, bb);
    if (bn >= 0.5f) {
      float brb[3] = {0.f, 0.f, 0.f};
      norm3_adj(braw, bb, brb);
      const float ndb = -dot3(n, brb);
      for (int i = 0; i < 3; i++) { z2b[i] += brb[i] + ndb * n[i]; nb[i] += -nd * brb[i] + ndb * z2[i]; }
    }
    for (int i = 0; i < 3; i++) { x2b[i] += spb[i]; z2b[i] += sg * h2 * spb[i]; z1b[i] += nb[i]; }
    return;
  }
  // closest points pa (on geom 1), pb (on geom 2), then sph_sph + make_frame
  float pa[3], pb[3];
  // forward intermediates of the capsule-capsule branch (kept for its adjoint)
  float a0[3], a1[3], b0[3], b1[3], dar[3], dbr[3], da[3], db[3], am[3], bm[3], tr[3];
  float la = 0.f, lb = 0.f, ha = 0.f, hb = 0.f, dadb = 0.f, datr = 0.f, dbtr = 0.f, den = 0.f, ta0 = 0.f, tb0 = 0.f;
  float ta = 0.f, tb = 0.f, pa0[3], pb0[3];
  bool use_na = false;
  if (kind == MJL_COL_SPHERE_SPHERE) {
    for (int i = 0; i < 3; i++) { pa[i] = x1[i]; pb[i] = x2[i]; }
  } else if (kind == MJL_COL_SPHERE_CAPSULE) {
    const float a[3] = {x2[0] - z2[0] * h2, x2[1] - z2[1] * h2, x2[2] - z2[2] * h2};
    const float bbv[3] = {x2[0] + z2[0] * h2, x2[1] + z2[1] * h2, x2[2] + z2[2] * h2};
    for (int i = 0; i < 3; i++) pa[i] = x1[i];
    seg_point(pb, a, bbv, x1);
  } else {
    for (int i = 0; i < 3; i++) {
      a0[i] = x1[i] - z1[i] * h1; a1[i] = x1[i] + z1[i] * h1;
      b0[i] = x2[i] - z2[i] * h2; b1[i] = x2[i] + z2[i] * h2;
      dar[i] = a1[i] - a0[i]; dbr[i] = b1[i] - b0[i]; da[i] = dar[i]; db[i] = dbr[i];
    }
    la = norm3(da); lb = norm3(db);
    ha = la * 0.5f; hb = lb * 0.5f;
    for (int i = 0; i < 3; i++) { am[i] = a0[i] + da[i] * ha; bm[i] = b0[i] + db[i] * hb; tr[i] = am[i] - bm[i]; }
    dadb = dot3(da, db); datr = dot3(da, tr); dbtr = dot3(db, tr);
    den = 1.f - dadb * dadb;
    ta0 = (-datr + dadb * dbtr) / (den + 1e-6f);
    tb0 = dbtr + ta0 * dadb;
    ta = fminf(fmaxf(ta0, -ha), ha); tb = fminf(fmaxf(tb0, -hb), hb);
    for (int i = 0; i < 3; i++) { pa0[i] = am[i] + da[i] * ta; pb0[i] = bm[i] + db[i] * tb; }
    float na[3], nb2[3];
    seg_point(na, a0, a1, pb0);
    seg_point(nb2, b0, b1, pa0);
    float d1 = 0.f, d2 = 0.f;
    for (int i = 0; i < 3; i++) { d1 += (pb0[i] - na[i]) * (pb0[i] - na[i]); d2 += (pa0[i] - nb2[i]) * (pa0[i] - nb2[i]); }
    use_na = d1 < d2;
    for (int i = 0; i < 3; i++) { pa[i] = use_na ? na[i] : pa0[i]; pb[i] = use_na ? pb0[i] : nb2[i]; }
  }
  // sph_sph + make_frame adjoint -> pa-bar, pb-bar
  float nraw[3] = {pb[0] - pa[0], pb[1] - pa[1], pb[2] - pa[2]}, n[3] = {nraw[0], nraw[1], nraw[2]};
  const float nrm = norm3(n);
  const float dist = nrm - (r1 + r2), s = r1 + dist * 0.5f;
  (void)dist;
  float nb[3] = {0.f, 0.f, 0.f}, pab[3] = {0.f, 0.f, 0.f}, pbb[3] = {0.f, 0.f, 0.f};
  make_frame_adj(n, frb, nb);
  for (int i = 0; i < 3; i++) { pab[i] += posb[i]; nb[i] += s * posb[i]; }
  distb += 0.5f * dot3(n, posb);
  float nrb[3] = {0.f, 0.f, 0.f};
  norm3_adj(nraw, nb, nrb);
  for (int i = 0; i < 3; i++) { nrb[i] += distb * n[i]; pbb[i] += nrb[i]; pab[i] -= nrb[i]; }
  if (kind == MJL_COL_SPHERE_SPHERE) {
    for (int i = 0; i < 3; i++) { x1b[i] += pab[i]; x2b[i] += pbb[i]; }
    return;
  }
  if (kind == MJL_COL_SPHERE_CAPSULE) {
    const float a[3] = {x2[0] - z2[0] * h2, x2[1] - z2[1] * h2, x2[2] - z2[2] * h2};
    const float bbv[3] = {x2[0] + z2[0] * h2, x2[1] + z2[1] * h2, x2[2] + z2[2] * h2};
    float aB[3] = {0.f, 0.f, 0.f}, bB[3] = {0.f, 0.f, 0.f};
    for (int i = 0; i < 3; i++) x1b[i] += pab[i];
    seg_point_adj(a, bbv, x1, pbb, aB, bB, x1b);
    for (int i = 0; i < 3; i++) { x2b[i] += aB[i] + bB[i]; z2b[i] += h2 * (bB[i] - aB[i]); }
    return;
  }
  // capsule-capsule (math.closest_segment_to_segment_points)
  float a0b[3] = {0.f, 0.f, 0.f}, a1b[3] = {0.f, 0.f, 0.f}, b0b[3] = {0.f, 0.f, 0.f}, b1b[3] = {0.f, 0.f, 0.f};
  float pa0b[3] = {0.f, 0.f, 0.f}, pb0b[3] = {0.f, 0.f, 0.f};
  if (use_na) {  // pa = seg_point(a0, a1, pb0), pb = pb0
    seg_point_adj(a0, a1, pb0, pab, a0b, a1b, pb0b);
    for (int i = 0; i < 3; i++) pb0b[i] += pbb[i];
  } else {       // pb = seg_point(b0, b1, pa0), pa = pa0
    seg_point_adj(b0, b1, pa0, pbb, b0b, b1b, pa0b);
    for (int i = 0; i < 3; i++) pa0b[i] += pab[i];
  }
  float amb[3], bmb[3], dab[3], dbb[3];
  for (int i = 0; i < 3; i++) { amb[i] = pa0b[i]; dab[i] = ta * pa0b[i]; bmb[i] = pb0b[i]; dbb[i] = tb * pb0b[i]; }
  float tab = dot3(da, pa0b), tbb = dot3(db, pb0b), hab = 0.f, hbb = 0.f;
  float tb0b = 0.f, ta0b = 0.f;
  if (tb0 > -hb && tb0 < hb) tb0b = tbb; else hbb += (tb0 >= hb ? 1.f : -1.f) * tbb;
  if (ta0 > -ha && ta0 < ha) ta0b = tab; else hab += (ta0 >= ha ? 1.f : -1.f) * tab;
  float dbtrb = tb0b, dadbb = tb0b * ta0;
  ta0b += tb0b * dadb;
  const float Q = den + 1e-6f, Nb = ta0b / Q, Qb = -ta0b * ta0 / Q;
  float datrb = -Nb;
  dadbb += Nb * dbtr;
  dbtrb += Nb * dadb;
  dadbb += -2.f * dadb * Qb;
  float trb[3];
  for (int i = 0; i < 3; i++) {
    dab[i] += dadbb * db[i] + datrb * tr[i];
    dbb[i] += dadbb * da[i] + dbtrb * tr[i];
    trb[i] = datrb * da[i] + dbtrb * db[i];
    amb[i] += trb[i]; bmb[i] -= trb[i];
  }
  for (int i = 0; i < 3; i++) { a0b[i] += amb[i]; dab[i] += ha * amb[i]; b0b[i] += bmb[i]; dbb[i] += hb * bmb[i]; }
  hab += dot3(da, amb); hbb += dot3(db, bmb);
  const float lab = 0.5f * hab, lbb = 0.5f * hbb;
  float darb[3] = {0.f, 0.f, 0.f}, dbrb[3] = {0.f, 0.f, 0.f};
  norm3_adj(dar, dab, darb);
  norm3_adj(dbr, dbb, dbrb);
  for (int i = 0; i < 3; i++) {
    darb[i] += lab * da[i]; dbrb[i] += lbb * db[i];
    a1b[i] += darb[i]; a0b[i] -= darb[i]; b1b[i] += dbrb[i]; b0b[i] -= dbrb[i];
    x1b[i] += a0b[i] + a1b[i]; z1b[i] += h1 * (a1b[i] - a0b[i]);
    x2b[i] += b0b[i] + b1b[i]; z2b[i] += h2 * (b1b[i] - b0b[i]);
  }
}

// lane = contact: geometry cotangents into the scratch record; then lane = geom gathers them
template <class D, class WT, class AT> INL void adj_collision(MP m, LDSA WT* W, LDSA AT* A, Rows<true> R, GLBA float* scr,
                                          int nefc_max, int lane) {
  const int ncon = W->ncon;
  GLBA float* conb = scr + 3 * nefc_max;
  for (int c = lane; c < ncon; c += 64) {
    GLBA float* cb = conb + c * kConAdjW;
    const int p = R.con_pair[c];
    const int k = (__float_as_int(R.con[c * CONW + 15]) >> 24) & 0xff;
    const PairRec pr = ldrec(&m->prec[p]);
    float posb[3] = {cb[0], cb[1], cb[2]}, frb[9];
    for (int i = 0; i < 9; i++) frb[i] = cb[3 + i];
    float x1b[3] = {0.f, 0.f, 0.f}, z1b[3] = {0.f, 0.f, 0.f}, x2b[3] = {0.f, 0.f, 0.f}, z2b[3] = {0.f, 0.f, 0.f};
    collide_adj<D>(pr, W, k, cb[12], posb, frb, x1b, z1b, x2b, z2b);
    for (int i = 0; i < 3; i++) { cb[13 + i] = x1b[i]; cb[16 + i] = z1b[i]; cb[19 + i] = x2b[i]; cb[22 + i] = z2b[i]; }
  }
  SYNC();
  if (lane < m->ngeom) {
    float gp[3] = {0.f, 0.f, 0.f}, ga[3] = {0.f, 0.f, 0.f};
    for (int c = 0; c < ncon; c++) {
      const PairRec pr = ldrec(&m->prec[R.con_pair[c]]);
      GLBA float* cb = conb + c * kConAdjW;
      if (pr.g1 == lane) for (int i = 0; i < 3; i++) { gp[i] += cb[13 + i]; ga[i] += cb[16 + i]; }
      if (pr.g2 == lane) for (int i = 0; i < 3; i++) { gp[i] += cb[19 + i]; ga[i] += cb[22 + i]; }
    }
    for (int i = 0; i < 3; i++) { A->gposb[lane][i] += gp[i]; A->gaxisb[lane][i] += ga[i]; }
  }
  SYNC();
}

// geom frames (kinematics): gpos = xpos_b + xmat_b geom_pos, gaxis = xmat_b zaxis; lane = body
template <class D, class AT> INL void adj_geom_frames(MP m, LDSA AT* A, int lane) {
  static_assert(D::NG <= D::NV, "geom constants staged in A->ftmp");
  // geom lanes stage their local pos / z axis (frame records) in A->ftmp, dead until adj_mass: the body
  // lanes' geom loop then reads LDS instead of waiting on two global loads per geom
  const bool isg = lane < m->ngeom;
  const uint32_t gmask = m->body_geommask[lane < m->nbody ? lane : 0];
  const FrameRec fr = ldrec(&m->frec[isg ? lane : 0]);
  if (isg)
    for (int j = 0; j < 3; j++) { A->ftmp[lane][j] = fr.pos[j]; A->ftmp[lane][3 + j] = fr.mat[j]; }
  SYNC();
  if (lane > 0 && lane < m->nbody) {
    for (uint32_t gm = gmask; gm; gm &= gm - 1) {
      const int g = __ffs(gm) - 1;
      for (int i = 0; i < 3; i++) {
        const float pb = A->gposb[g][i], ab = A->gaxisb[g][i];
        A->xposb[lane][i] += pb;
        for (int j = 0; j < 3; j++) A->xmatb[lane][3 * i + j] += pb * A->ftmp[g][j] + ab * A->ftmp[g][3 + j];
      }
    }
  }
  SYNC();
}

// qfrc_smooth = passive - bias + actuator: passive and actuation adjoints; bias-bar -> A->vtmp
template <class D, class WT, class AT> INL void adj_forces(MP m, LDSA WT* W, LDSA AT* A, int lane) {
  const int nv = m->nv, nu = m->nu;
  const int ul = lane < nu ? lane : 0;  // actuator constants issued with the dof record
  const int a_lim = m->actuator_ctrllimited[ul], a_dof = m->actuator_dof[ul];
  const float a_lo = m->actuator_ctrlrange[ul][0], a_hi = m->actuator_ctrlrange[ul][1], a_gear = m->actuator_gear[ul];
  const DofRec dr = ldrec(&m->drec[lane < nv ? lane : 0]);
  if (lane < nv) {
    const float fs = A->frcsb[lane];
    A->vtmp[lane] = -fs;
    A->frcactb[lane] += fs;
    A->qvelb[lane] += -dr.damping * fs;
    if (dr.qadr_spring >= 0) A->qposb[dr.qadr_spring] += -dr.stiffness * fs;
  }
  SYNC();
  if (lane < nu) {
    const float c = W->ctrl[lane];
    const bool inside = !a_lim || (c > a_lo && c < a_hi);
    A->ctrlb[lane] += inside ? a_gear * A->frcactb[a_dof] : 0.f;
  }
  SYNC();
}

// per-body velocity terms (velocity_stage): S, U, T from cdof and qvel
template <class D, class WT> INL void body_vel_terms(LDSA WT* W, const LDSA float* qvel, const BodyRec& br, float* S,
                                           float* U, float* T) {
  for (int i = 0; i < 6; i++) { S[i] = 0.f; U[i] = 0.f; T[i] = 0.f; }
  const int da = br.dofadr, dn = br.dofnum;
  if (br.isfree) {
    for (int k = 0; k < 3; k++)
      for (int i = 0; i < 6; i++) S[i] += W->cdof[da + k][i] * qvel[da + k];
    for (int k = 3; k < 6; k++)
      for (int i = 0; i < 6; i++) U[i] += W->cdof[da + k][i] * qvel[da + k];
    cross_motion(T, S, U);
    for (int i = 0; i < 6; i++) S[i] += U[i];
  } else {
    for (int k = 0; k < dn; k++) {
      float v[6], x[6];
      for (int i = 0; i < 6; i++) v[i] = W->cdof[da + k][i] * qvel[da + k];
      cross_motion(x, S, v);
      for (int i = 0; i < 6; i++) { T[i] += x[i]; U[i] += v[i]; S[i] += v[i]; }
    }
  }
}

// recursive Newton-Euler (qfrc_bias) adjoint. In: bias-bar in A->vtmp. W->cvel holds the
// subtree force sums, W->cacc the body forces (velocity_stage overwrote them).
template <class D, class WT, class AT> INL void adj_rne(MP m, LDSA WT* W, LDSA AT* A, int lane) {
  const int nv = m->nv, nbody = m->nbody, maxlevel = m->maxlevel;
  const bool isb = lane > 0 && lane < nbody;
  const int bl = lane < nbody ? lane : 0;  // the pass's model records, issued together
  const BodyRec br = ldrec(&m->brec[isb ? lane : 0]);
  const int dbody = ldrec(&m->drec[lane < nv ? lane : 0]).bodyid;
  const uint32_t ancm = m->body_ancmask[bl], chm = m->body_childmask[bl];
  TSTART(tr);
  if (lane < nv) {  // bias_d = cdof_d . cfsub_body(d)
    const int b = dbody;
    for (int k = 0; k < 6; k++) A->cdofb[lane][k] += A->vtmp[lane] * W->cvel[b][k];
  }
  if (isb) {
    float s[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int d = br.dofadr; d < br.dofadr + br.dofnum; d++)
      for (int k = 0; k < 6; k++) s[k] += A->vtmp[d] * W->cdof[d][k];
    for (int k = 0; k < 6; k++) A->cfsubb[lane][k] = s[k];
  }
  SYNC();
  if (isb) {  // cfrc-bar_c = sum over ancestors-or-self b of cfsub-bar_b
    float s[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (uint32_t mk = ancm; mk;) {  // self, then up the chain
      const int b = 31 - __clz(mk);
      mk &= ~(1u << b);
      for (int k = 0; k < 6; k++) s[k] += A->cfsubb[b][k];
    }
    for (int k = 0; k < 6; k++) A->cfrcb[lane][k] = s[k];
  }
  TACC(25, tr, lane);
  // recompute cvel / cacc (tree pass of velocity_stage) level by level in registers: each body lane
  // pulls its parent's values by lane shuffle (every lane takes part), no LDS round trip or barrier
  float S[6], U[6], T[6];
  if (isb) body_vel_terms<D>(W, A->qvel0, br, S, U, T);
  float cv[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float ca[6] = {0.f, 0.f, 0.f, -m->gravity[0], -m->gravity[1], -m->gravity[2]};  // the world's (lane 0)
  const int par = isb ? br.parent : 0;
  for (int L = 1; L <= maxlevel; L++) {
    float pv[6], pa[6];
    for (int i = 0; i < 6; i++) { pv[i] = __shfl(cv[i], par); pa[i] = __shfl(ca[i], par); }
    if (isb && br.level == L) {
      float x[6];
      cross_motion(x, pv, U);
      for (int i = 0; i < 6; i++) { cv[i] = pv[i] + S[i]; ca[i] = pa[i] + x[i] + T[i]; }
    }
  }
  float pcv[6];  // the parent's cvel, for the tree reverse
  for (int i = 0; i < 6; i++) pcv[i] = __shfl(cv[i], par);
  TACC(26, tr, lane);
  // cfrc = I cacc + cvel x* (I cvel); the cvel / cacc cotangent accumulators stay in registers
  float cvacc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, caacc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (isb) {
    float ci[10], fb[6], iv[6], ivb[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float cib[10] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, cvb[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float cab[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < 10; i++) ci[i] = W->cinert[lane][i];
    for (int i = 0; i < 6; i++) fb[i] = A->cfrcb[lane][i];
    inert_vec(iv, ci, cv);
    inert_vec_adj(ci, ca, fb, cib, cab);
    cross_force_adj(cv, iv, fb, cvb, ivb);
    inert_vec_adj(ci, cv, ivb, cib, cvb);
    for (int i = 0; i < 10; i++) A->cinertb[lane][i] += cib[i];
    for (int i = 0; i < 6; i++) { cvacc[i] = 0.f + cvb[i]; caacc[i] = 0.f + cab[i]; }
  }
  SYNC();
  TACC(27, tr, lane);
  // tree reverse: cvel_b = cvel_p + S, cacc_b = cacc_p + cvel_p x U + T; children -> parent gather
  // through each body's own cfsubb / cfrcb row (written once, at its level: one barrier per level)
  float Sb[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, Ubr[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, Tbr[6];
  for (int L = maxlevel; L >= 1; L--) {
    if (isb && br.level == L) {
      float pvb[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int i = 0; i < 6; i++) { Sb[i] = cvacc[i]; Tbr[i] = caacc[i]; }
      cross_motion_adj(pcv, U, Tbr, pvb, Ubr);
      for (int i = 0; i < 6; i++) { A->cfsubb[lane][i] = Sb[i] + pvb[i]; A->cfrcb[lane][i] = Tbr[i]; }
    }
    SYNC();
    if (isb && br.level == L - 1) {
      for (uint32_t mk = chm; mk; mk &= mk - 1) {
        const int c = __ffs(mk) - 1;
        for (int i = 0; i < 6; i++) { cvacc[i] += A->cfsubb[c][i]; caacc[i] += A->cfrcb[c][i]; }
      }
    }
  }
  SYNC();
  TACC(28, tr, lane);
  if (isb) {  // local terms -> cdof-bar, qvel-bar
    const int da = br.dofadr, dn = br.dofnum;
    if (br.isfree) {
      float St[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, Uf[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int k = 0; k < 3; k++)
        for (int i = 0; i < 6; i++) St[i] += W->cdof[da + k][i] * A->qvel0[da + k];
      for (int k = 3; k < 6; k++)
        for (int i = 0; i < 6; i++) Uf[i] += W->cdof[da + k][i] * A->qvel0[da + k];
      float Stb[6], Utb[6];
      for (int i = 0; i < 6; i++) { Stb[i] = Sb[i]; Utb[i] = Ubr[i] + Sb[i]; }
      cross_motion_adj(St, Uf, Tbr, Stb, Utb);
      for (int k = 0; k < 6; k++) {
        const int d = da + k;
        const float* vb = k < 3 ? Stb : Utb;
        float dot = 0.f;
        for (int i = 0; i < 6; i++) { A->cdofb[d][i] += A->qvel0[d] * vb[i]; dot += W->cdof[d][i] * vb[i]; }
        A->qvelb[d] += dot;
      }
    } else {
      float Srun[6];
      for (int i = 0; i < 6; i++) Srun[i] = Sb[i];
      for (int k = dn - 1; k >= 0; k--) {
        float Sk[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, v[6];
        for (int kk = 0; kk < k; kk++)
          for (int i = 0; i < 6; i++) Sk[i] += W->cdof[da + kk][i] * A->qvel0[da + kk];
        const int d = da + k;
        for (int i = 0; i < 6; i++) v[i] = W->cdof[d][i] * A->qvel0[d];
        float skb[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, vb[6];
        for (int i = 0; i < 6; i++) vb[i] = Srun[i] + Ubr[i];
        cross_motion_adj(Sk, v, Tbr, skb, vb);
        for (int i = 0; i < 6; i++) Srun[i] += skb[i];
        float dot = 0.f;
        for (int i = 0; i < 6; i++) { A->cdofb[d][i] += A->qvel0[d] * vb[i]; dot += W->cdof[d][i] * vb[i]; }
        A->qvelb[d] += dot;
      }
    }
  }
  SYNC();
  TACC(29, tr, lane);
}

// mass matrix (crb / make_m): M[i][j] = cdof_j . I(crb_body(i)) cdof_i (+ armature), j in anc(i)
template <class D, class WT, class AT, class MT>
INL void adj_mass(MP m, LDSA WT* W, LDSA AT* A, const MT& mt, bool unr, int lane) {
  constexpr int LD = D::LD;
  const int nv = m->nv;
  const bool isd = lane < nv;
  const DofRec dr = ldrec(&m->drec[isd ? lane : 0]);
  const uint32_t descm = m->dof_descmask[isd ? lane : 0];
  const BodyRec brm = ldrec(&m->brec[lane > 0 && lane < m->nbody ? lane : 0]);  // the crb-bar pass below
  // M-bar[i][j]: the accumulated array, or (lean replay) its rank-one terms in the order and form the
  // array accumulated them: adj_integrate's rb (qacc - a')^T (damped implicit / eulerdamp), then
  // adj_solver_rows' -mu qacc^T, each a fused multiply-add onto the running value from 0
  const bool damp = (m->integrator == MJL_INT_IMPLICITFAST || m->eulerdamp) && m->any_damping;
  TSTART(tm);
  if (isd) {
    float f6[6];
    inert_vec(f6, W->crb[dr.bodyid], W->cdof[lane]);
    for (int k = 0; k < 6; k++) A->ftmp[lane][k] = f6[k];
  }
  if constexpr (is_lean<AT>::value) {  // M-bar's rank-one operands packed per dof: one b128 read per (i, j)
    if (lane < LD) {
      f32x4 v;
      v[0] = A->mu[lane]; v[1] = A->rb[lane]; v[2] = W->qacc[lane]; v[3] = A->ap[lane];
      ((LDSA f32x4*)A->mq)[lane] = v;
    }
  }
  SYNC();
  float fb[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // the loops, instantiated per M-bar source (the choice made once, outside them)
  auto loops = [&](auto mbar) {
    const int i = lane;
    for (uint32_t anc = dr.ancmask; anc;) {  // f-bar_i = sum_j vbar_ij cdof_j
      const int j = 31 - __builtin_clz(anc);
      anc &= ~(1u << j);
      const float vb = (j == i) ? mbar(i, i) : mbar(i, j) + mbar(j, i);
      for (int k = 0; k < 6; k++) fb[k] += vb * W->cdof[j][k];
    }
    const int j = lane;  // cdof-bar_j += sum over descendants i of vbar_ij f_i
    // every dof in ascending order, the sum taking the descendants (the mask's bit loop, unrolled:
    // a root dof has all nv as descendants, and the loop waited for each iteration's LDS reads)
    float cb[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll  // (fully: 98.6 against 99.7 us per replay unrolled by 9)
    for (int ii = 0; ii < D::NV; ii++) {
      const bool in = (descm >> ii) & 1u;
      const float a = mbar(ii, j), c = mbar(j, ii);
      const float vb = (ii == j) ? c : a + c;
      float f[6];
      for (int k = 0; k < 6; k++) f[k] = A->ftmp[ii][k];
      for (int k = 0; k < 6; k++) cb[k] = in ? cb[k] + vb * f[k] : cb[k];
    }
    for (int k = 0; k < 6; k++) A->cdofb[j][k] += cb[k];
  };
  if (isd) {
    if constexpr (is_lean<AT>::value) {
      if (unr) {  // unrolled: the rows adj_solver_unrolled accumulated
        loops([&](int i, int j) -> float { return mt.Mb[i * LD + j]; });
      } else if (damp) {
        loops([&](int i, int j) -> float {
          const f32x4 a = ((const LDSA f32x4*)A->mq)[i], b = ((const LDSA f32x4*)A->mq)[j];
          return fmaf(-a[0], b[2], fmaf(a[1], b[2] - b[3], 0.f));
        });
      } else {
        loops([&](int i, int j) -> float {
          const f32x4 a = ((const LDSA f32x4*)A->mq)[i], b = ((const LDSA f32x4*)A->mq)[j];
          return fmaf(-a[0], b[2], 0.f);
        });
      }
    } else {
      loops([&](int i, int j) -> float { return A->Mb[i * LD + j]; });
    }
  }
  SYNC();
  TACC(30, tm, lane);
  if (isd) {  // f_i = I(crb) cdof_i
    float t[6];
    inert_vec(t, W->crb[dr.bodyid], fb);
    for (int k = 0; k < 6; k++) { A->cdofb[lane][k] += t[k]; A->ftmp[lane][k] = fb[k]; }
  }
  SYNC();
  if (lane > 0 && lane < m->nbody) {
    const BodyRec& br = brm;
    float ib[10] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int d = br.dofadr; d < br.dofadr + br.dofnum; d++) {
      float f6[6], c6[6];
      for (int k = 0; k < 6; k++) { f6[k] = A->ftmp[d][k]; c6[k] = W->cdof[d][k]; }
      inert_vec_adj(W->crb[lane], c6, f6, ib, (float*)nullptr);
    }
    for (int k = 0; k < 10; k++) A->crbb[lane][k] += ib[k];
  }
  SYNC();
  TACC(31, tm, lane);
}

// crb_b = sum of cinert over the subtree of b: cinert-bar_c = sum of crb-bar over ancestors-or-self
template <class D, class AT> INL void adj_crb(MP m, LDSA AT* A, int lane) {
  if (lane > 0 && lane < m->nbody) {
    float s[10] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (uint32_t mk = m->body_ancmask[lane]; mk;) {  // self, then up the chain
      const int b = 31 - __clz(mk);
      mk &= ~(1u << b);
      for (int k = 0; k < 10; k++) s[k] += A->crbb[b][k];
    }
    for (int k = 0; k < 10; k++) A->cinertb[lane][k] += s[k];
  }
  SYNC();
}

// cinert (com_pos): rotated inertia about the root's subtree com -> xmat, xipos, scom
template <class D, class WT, class AT> INL void adj_cinert(MP m, LDSA WT* W, LDSA AT* A, int lane) {
  const bool isb = lane > 0 && lane < m->nbody;
  const BodyRec br = ldrec(&m->brec[isb ? lane : 0]);
  float scb[3] = {0.f, 0.f, 0.f};
  if (isb && br.mass != 0.f) {
    const int b = lane, root = br.rootid;
    const float ms = br.mass;
    LDSA float* cb = A->cinertb[b];
    const float* t = br.inertia;  // body_inertia[b], in the record
    const float Ib[9] = {t[0], t[3], t[4], t[3], t[1], t[5], t[4], t[5], t[2]};
    float X[9];
    for (int i = 0; i < 9; i++) X[i] = W->xmat[b][i];
    float G[9] = {cb[0], cb[3], cb[4], 0.f, cb[1], cb[5], 0.f, 0.f, cb[2]};
    float S[9];  // G + G^T
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) S[3 * i + j] = G[3 * i + j] + G[3 * j + i];
    float XI[9];  // X Ib
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) XI[3 * i + j] = X[3 * i] * Ib[j] + X[3 * i + 1] * Ib[3 + j] + X[3 * i + 2] * Ib[6 + j];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++)
        A->xmatb[b][3 * i + j] += S[3 * i] * XI[j] + S[3 * i + 1] * XI[3 + j] + S[3 * i + 2] * XI[6 + j];
    const float c[3] = {W->xipos[b][0] - W->scom[root][0], W->xipos[b][1] - W->scom[root][1],
                        W->xipos[b][2] - W->scom[root][2]};
    float cbar[3];
    for (int i = 0; i < 3; i++) cbar[i] = 2.f * ms * c[i] * (cb[0] + cb[1] + cb[2]) + ms * cb[6 + i];
    cbar[0] -= 2.f * ms * c[0] * cb[0]; cbar[1] -= 2.f * ms * c[1] * cb[1]; cbar[2] -= 2.f * ms * c[2] * cb[2];
    cbar[0] -= ms * (cb[3] * c[1] + cb[4] * c[2]);
    cbar[1] -= ms * (cb[3] * c[0] + cb[5] * c[2]);
    cbar[2] -= ms * (cb[4] * c[0] + cb[5] * c[1]);
    for (int i = 0; i < 3; i++) { A->xiposb[b][i] += cbar[i]; scb[i] = -cbar[i]; }
  }
  scom_reduce<D>(m, A, isb ? br.rootid : -1, scb, lane);
  SYNC();
}

// cdof (com_pos): hinge (axis, axis x (scom_root - anchor)); free rotation uses xmat columns
template <class D, class WT, class AT> INL void adj_cdof(MP m, LDSA WT* W, LDSA AT* A, int lane) {
  const int nv = m->nv;
  const bool isd = lane < nv;
  const DofRec dr = ldrec(&m->drec[isd ? lane : 0]);
  const JntRec jown = ldrec(&m->jrec[lane < m->njnt ? lane : 0]);  // the joint gather below
  float scb[3] = {0.f, 0.f, 0.f};
  if (isd) {
    const int d = lane, j = dr.jntid, b = dr.bodyid, root = dr.rootid, k = dr.kfree;
    float axb[3] = {0.f, 0.f, 0.f}, offb[3] = {0.f, 0.f, 0.f};
    if (!(k >= 0 && k < 3)) {
      float ax[3];
      if (k >= 3) { ax[0] = W->xmat[b][k - 3]; ax[1] = W->xmat[b][3 + k - 3]; ax[2] = W->xmat[b][6 + k - 3]; }
      else { ax[0] = W->xaxis[j][0]; ax[1] = W->xaxis[j][1]; ax[2] = W->xaxis[j][2]; }
      const float off[3] = {W->scom[root][0] - W->xanchor[j][0], W->scom[root][1] - W->xanchor[j][1],
                            W->scom[root][2] - W->xanchor[j][2]};
      float lb[3] = {A->cdofb[d][3], A->cdofb[d][4], A->cdofb[d][5]};
      axb[0] = A->cdofb[d][0]; axb[1] = A->cdofb[d][1]; axb[2] = A->cdofb[d][2];
      cross3_adj(ax, off, lb, axb, offb);
      for (int i = 0; i < 3; i++) scb[i] = offb[i];
    }
    for (int i = 0; i < 3; i++) { A->ftmp[d][i] = axb[i]; A->ftmp[d][3 + i] = offb[i]; }
  }
  scom_reduce<D>(m, A, isd ? dr.rootid : -1, scb, lane);
  SYNC();
  if (lane < m->njnt) {  // gather the joint's dofs
    const JntRec& jr = jown;
    const int nd = jr.isfree ? 6 : 1;
    for (int q = 0; q < nd; q++) {
      const int d = jr.dofadr + q;
      for (int i = 0; i < 3; i++) A->xanchorb[lane][i] -= A->ftmp[d][3 + i];
      if (!jr.isfree) for (int i = 0; i < 3; i++) A->xaxisb[lane][i] += A->ftmp[d][i];
      else if (q >= 3) for (int i = 0; i < 3; i++) A->xmatb[jr.body][3 * i + (q - 3)] += A->ftmp[d][i];
    }
  }
  SYNC();
}

// kinematics: root subtree com, joint frames, xipos, the level-by-level tree pass, and the
// per-body local transforms -> qpos-bar
template <class D, class WT, class AT> INL void adj_kinematics(MP m, LDSA WT* W, LDSA AT* A, int lane) {
  const int nbody = m->nbody, maxlevel = m->maxlevel, njnt = m->njnt;
  const bool isb = lane > 0 && lane < nbody;
  // the pass's model records issued together up front (the loops below waited on one dependent
  // record load per joint: ~10 global round trips per env): the lane's body and joint, its masks and
  // root mass, then the body's first three hinges (one more round, through jntadr)
  const int bl = lane < nbody ? lane : 0;
  const BodyRec br = ldrec(&m->brec[isb ? lane : 0]);
  const JntRec jown = ldrec(&m->jrec[lane < njnt ? lane : 0]);
  const uint32_t jgather = m->body_jgather[bl], cmask_nf = m->body_childmask_nf[bl];
  const float rmass_own = m->body_rootmass[bl];
  const int ja = isb && br.jntadr >= 0 ? br.jntadr : 0;
  const JntRec bj0 = ldrec(&m->jrec[ja < njnt ? ja : 0]);
  const JntRec bj1 = ldrec(&m->jrec[ja + 1 < njnt ? ja + 1 : 0]);
  const JntRec bj2 = ldrec(&m->jrec[ja + 2 < njnt ? ja + 2 : 0]);
  auto hinge = [&](int q) -> JntRec {
    if (q < 3) return q == 0 ? bj0 : (q == 1 ? bj1 : bj2);
    return ldrec(&m->jrec[br.jntadr + q]);
  };
  TSTART(tk);
  const uint64_t freemask = __ballot(lane < njnt && jown.isfree);  // bit j: joint j is free
  const float mr = __shfl(rmass_own, isb ? br.rootid : 0);         // body_rootmass[rootid]
  // scom_r = sum_c m_c xipos_c / sum_c m_c over the root's subtree
  if (isb) {
    const int r = br.rootid;
    if (mr >= kMinVal) for (int i = 0; i < 3; i++) A->xiposb[lane][i] += br.mass / mr * A->scomb[r][i];
  }
  SYNC();
  // joint anchors / axes (world) -> parent frame cotangents; local anchor / axis cotangents in ftmp
  if (lane < njnt) {
    const JntRec& jr = jown;
    if (!jr.isfree) {
      const int p = jr.parent;
      float lab[3], lxb[3];
      mtv3(lab, W->xmat[p], A->xanchorb[lane]);
      mtv3(lxb, W->xmat[p], A->xaxisb[lane]);
      for (int i = 0; i < 3; i++) { A->ftmp[lane][i] = lab[i]; A->ftmp[lane][3 + i] = lxb[i]; }
    }
  }
  SYNC();
  TACC(20, tk, lane);
  if (lane < nbody) {  // gather: free joint -> its body; hinge -> its parent frame (la, lx in local)
    float pb[3] = {0.f, 0.f, 0.f}, mb[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (uint32_t mk = jgather; mk; mk &= mk - 1) {
      const int j = __ffs(mk) - 1;
      if ((freemask >> j) & 1ull) {
        for (int i = 0; i < 3; i++) { pb[i] += A->xanchorb[j][i]; mb[3 * i + 2] += A->xaxisb[j][i]; }
      } else {
        // anc = xpos_p + xmat_p la, ax = xmat_p lx with la, lx the local values stored in xanchor/xaxis?
        // (the forward overwrote them with world values: recover local = xmat_p^T (world - xpos_p))
        float la[3], lx[3], wa[3] = {W->xanchor[j][0] - W->xpos[lane][0], W->xanchor[j][1] - W->xpos[lane][1],
                                     W->xanchor[j][2] - W->xpos[lane][2]};
        mtv3(la, W->xmat[lane], wa);
        mtv3(lx, W->xmat[lane], W->xaxis[j]);
        for (int i = 0; i < 3; i++) {
          pb[i] += A->xanchorb[j][i];
          for (int k = 0; k < 3; k++) mb[3 * i + k] += A->xanchorb[j][i] * la[k] + A->xaxisb[j][i] * lx[k];
        }
      }
    }
    for (int i = 0; i < 3; i++) A->xposb[lane][i] += pb[i];
    for (int i = 0; i < 9; i++) A->xmatb[lane][i] += mb[i];
  }
  SYNC();
  TACC(21, tk, lane);
  if (isb) {  // xipos = xpos + xmat ipos
    for (int i = 0; i < 3; i++) {
      A->xposb[lane][i] += A->xiposb[lane][i];
      for (int k = 0; k < 3; k++) A->xmatb[lane][3 * i + k] += A->xiposb[lane][i] * br.ipos[k];
    }
  }
  // local transforms (as the forward computes them), kept in A->lp / A->lq; the first three hinges'
  // intermediates (quaternion before the joint, sin / cos of its half angle) stay in registers for
  // the reverse below, which recomputed the chain
  float kq[3][4], ks[3], kc[3];
  if (isb) {
    float lp[3], lq[4];
    if (br.isfree) {
      const int qa = br.qadr;
      for (int i = 0; i < 3; i++) lp[i] = A->qpos0[qa + i];
      for (int i = 0; i < 4; i++) lq[i] = A->qpos0[qa + 3 + i];
      qnorm(lq);
    } else {
      for (int i = 0; i < 3; i++) lp[i] = br.pos[i];
      for (int i = 0; i < 4; i++) lq[i] = br.quat[i];
      auto joint = [&](int q, float& s, float& c) {
        const JntRec jr = hinge(q);
        float mat[9], anc[3], off[3];
        q2m(mat, lq);
        mv3(anc, mat, jr.pos);
        for (int i = 0; i < 3; i++) anc[i] += lp[i];
        sincosf(0.5f * (A->qpos0[jr.qadr] - jr.qpos0), &s, &c);
        const float ql[4] = {c, jr.axis[0] * s, jr.axis[1] * s, jr.axis[2] * s};
        qmul(lq, lq, ql);
        q2m(mat, lq);
        mv3(off, mat, jr.pos);
        for (int i = 0; i < 3; i++) lp[i] = anc[i] - off[i];
      };
      const int jn = br.jntnum;
#pragma unroll
      for (int q = 0; q < 3; q++) {
        if (q < jn) {
          for (int i = 0; i < 4; i++) kq[q][i] = lq[i];
          joint(q, ks[q], kc[q]);
        }
      }
      for (int q = 3; q < jn; q++) {
        float s, c;
        joint(q, s, c);
      }
    }
    for (int i = 0; i < 3; i++) A->lp[lane][i] = lp[i];
    for (int i = 0; i < 4; i++) A->lq[lane][i] = lq[i];
  }
  SYNC();
  TACC(22, tk, lane);
  // tree pass reverse; child contributions to the parent go through A->Sb (xquat 4, xpos 3) and
  // A->Tb (first 6 of xmat) + A->Ub (last 3 of xmat). The body's cotangent accumulators (xquat, xpos,
  // xmat) live in its lane's registers through the level loop (its children's contributions are added
  // there), and the forward-only operands (its and its parent's frames, the local transform, the
  // pre-normalisation quaternion and its norm) are loaded / formed once before the loop: each level's
  // chain is then the cotangent arithmetic and one LDS exchange with one barrier (each body writes
  // only its own Sb / Tb / Ub row, once, so no second barrier protects them).
  float lpb[3] = {0.f, 0.f, 0.f}, lqb[4] = {0.f, 0.f, 0.f, 0.f};
  float qacc[4] = {0.f, 0.f, 0.f, 0.f}, pacc[3] = {0.f, 0.f, 0.f};
  float macc[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float xqb[4] = {1.f, 0.f, 0.f, 0.f}, xqp[4] = {1.f, 0.f, 0.f, 0.f}, lqv[4] = {1.f, 0.f, 0.f, 0.f};
  float xmp[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, lpv[3] = {0.f, 0.f, 0.f};
  float qn[4] = {0.f, 0.f, 0.f, 0.f}, qinv = 0.f;
  bool qok = false;
  if (isb) {
    for (int i = 0; i < 4; i++) { qacc[i] = A->xquatb[lane][i]; xqb[i] = W->xquat[lane][i]; }
    for (int i = 0; i < 3; i++) pacc[i] = A->xposb[lane][i];
    for (int i = 0; i < 9; i++) macc[i] = A->xmatb[lane][i];
    if (!br.isfree) {
      const int p = br.parent;
      for (int i = 0; i < 4; i++) { xqp[i] = W->xquat[p][i]; lqv[i] = A->lq[lane][i]; }
      for (int i = 0; i < 9; i++) xmp[i] = W->xmat[p][i];
      for (int i = 0; i < 3; i++) lpv[i] = A->lp[lane][i];
      float pre[4];
      qmul(pre, xqp, lqv);
      const float n = sqrtf(pre[0] * pre[0] + pre[1] * pre[1] + pre[2] * pre[2] + pre[3] * pre[3]);  // qnorm_adj
      qok = !(n < kMinVal);
      qinv = 1.f / n;
      for (int i = 0; i < 4; i++) qn[i] = pre[i] * qinv;
    }
  }
  for (int L = maxlevel; L >= 1; L--) {
    if (isb && br.level == L) {
      const int b = lane;
      float qb[4] = {qacc[0], qacc[1], qacc[2], qacc[3]};
      q2m_adj(xqb, macc, qb);
      float cq[4] = {0.f, 0.f, 0.f, 0.f}, cp[3] = {0.f, 0.f, 0.f}, cm[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (br.isfree) {
        for (int i = 0; i < 3; i++) lpb[i] = pacc[i];
        for (int i = 0; i < 4; i++) lqb[i] = qb[i];
      } else {
        float preb[4] = {0.f, 0.f, 0.f, 0.f};
        if (qok) {  // qnorm_adj(pre, qb, preb) with the forward's part formed above
          const float d = qn[0] * qb[0] + qn[1] * qb[1] + qn[2] * qb[2] + qn[3] * qb[3];
          for (int i = 0; i < 4; i++) preb[i] += (qb[i] - qn[i] * d) * qinv;
        }
        qmul_adj(xqp, lqv, preb, cq, lqb);
        for (int i = 0; i < 3; i++) cp[i] = pacc[i];
        mv3_adj(xmp, lpv, pacc, cm, lpb);
      }
      for (int i = 0; i < 4; i++) A->Sb[b][i] = cq[i];
      for (int i = 0; i < 2; i++) A->Sb[b][4 + i] = cp[i];
      A->Ub[b][0] = cp[2];
      for (int i = 0; i < 6; i++) A->Tb[b][i] = cm[i];
      for (int i = 0; i < 3; i++) A->Ub[b][1 + i] = cm[6 + i];
    }
    SYNC();
    if (isb && br.level == L - 1) {
      for (uint32_t mk = cmask_nf; mk; mk &= mk - 1) {
        const int c = __ffs(mk) - 1;
        for (int i = 0; i < 4; i++) qacc[i] += A->Sb[c][i];
        pacc[0] += A->Sb[c][4]; pacc[1] += A->Sb[c][5]; pacc[2] += A->Ub[c][0];
        for (int i = 0; i < 6; i++) macc[i] += A->Tb[c][i];
        for (int i = 0; i < 3; i++) macc[6 + i] += A->Ub[c][1 + i];
      }
    }
  }
  SYNC();
  TACC(23, tk, lane);
  // local transforms reverse -> qpos-bar
  if (isb) {
    if (br.isfree) {
      const int qa = br.qadr;
      for (int i = 0; i < 3; i++) A->qposb[qa + i] += lpb[i];
      const float q[4] = {A->qpos0[qa + 3], A->qpos0[qa + 4], A->qpos0[qa + 5], A->qpos0[qa + 6]};
      float qb[4] = {0.f, 0.f, 0.f, 0.f};
      qnorm_adj(q, lqb, qb);
      for (int i = 0; i < 4; i++) A->qposb[qa + 3 + i] += qb[i];
    } else if (br.jntnum <= 3) {  // the intermediates cached above
#pragma unroll
      for (int q = 2; q >= 0; q--) {
        if (q < br.jntnum) {
          const int j = br.jntadr + q;
          const JntRec jr = hinge(q);
          const float ql[4] = {kc[q], jr.axis[0] * ks[q], jr.axis[1] * ks[q], jr.axis[2] * ks[q]};
          float lqa[4];
          qmul(lqa, kq[q], ql);
          float ancb[3] = {lpb[0], lpb[1], lpb[2]};
          float m2b[9];
          for (int i = 0; i < 3; i++)
            for (int k = 0; k < 3; k++) m2b[3 * i + k] = -lpb[i] * jr.pos[k];
          q2m_adj(lqa, m2b, lqb);
          float lqbb[4] = {0.f, 0.f, 0.f, 0.f}, qlb[4] = {0.f, 0.f, 0.f, 0.f};
          qmul_adj(kq[q], ql, lqb, lqbb, qlb);
          const float thb = -ks[q] * qlb[0] + kc[q] * (jr.axis[0] * qlb[1] + jr.axis[1] * qlb[2] + jr.axis[2] * qlb[3]);
          A->qposb[jr.qadr] += 0.5f * thb;
          for (int i = 0; i < 3; i++) ancb[i] += A->ftmp[j][i];
          float mb[9];
          for (int i = 0; i < 3; i++)
            for (int k = 0; k < 3; k++) mb[3 * i + k] = ancb[i] * jr.pos[k] + A->ftmp[j][3 + i] * jr.axis[k];
          q2m_adj(kq[q], mb, lqbb);
          for (int i = 0; i < 3; i++) lpb[i] = ancb[i];
          for (int i = 0; i < 4; i++) lqb[i] = lqbb[i];
        }
      }
    } else {
      constexpr int KJ = 8;  // joints per body kept for the reverse sweep
      float lqs[KJ][4], lps[KJ][3], sn[KJ], cs[KJ];
      float lp[3], lq[4];
      for (int i = 0; i < 3; i++) lp[i] = br.pos[i];
      for (int i = 0; i < 4; i++) lq[i] = br.quat[i];
      const int jn = br.jntnum < KJ ? br.jntnum : KJ;
      for (int q = 0; q < jn; q++) {
        const JntRec jr = hinge(q);
        for (int i = 0; i < 4; i++) lqs[q][i] = lq[i];
        for (int i = 0; i < 3; i++) lps[q][i] = lp[i];
        float mat[9], anc[3], off[3];
        q2m(mat, lq);
        mv3(anc, mat, jr.pos);
        for (int i = 0; i < 3; i++) anc[i] += lp[i];
        sincosf(0.5f * (A->qpos0[jr.qadr] - jr.qpos0), &sn[q], &cs[q]);
        const float ql[4] = {cs[q], jr.axis[0] * sn[q], jr.axis[1] * sn[q], jr.axis[2] * sn[q]};
        qmul(lq, lq, ql);
        q2m(mat, lq);
        mv3(off, mat, jr.pos);
        for (int i = 0; i < 3; i++) lp[i] = anc[i] - off[i];
      }
      for (int q = jn - 1; q >= 0; q--) {
        const int j = br.jntadr + q;
        const JntRec jr = hinge(q);
        const float ql[4] = {cs[q], jr.axis[0] * sn[q], jr.axis[1] * sn[q], jr.axis[2] * sn[q]};
        float lqa[4];
        qmul(lqa, lqs[q], ql);
        // lp_after = anc - q2m(lq_after) jpos
        float ancb[3] = {lpb[0], lpb[1], lpb[2]};
        float m2b[9];
        for (int i = 0; i < 3; i++)
          for (int k = 0; k < 3; k++) m2b[3 * i + k] = -lpb[i] * jr.pos[k];
        q2m_adj(lqa, m2b, lqb);
        // lq_after = lq_before (x) ql
        float lqbb[4] = {0.f, 0.f, 0.f, 0.f}, qlb[4] = {0.f, 0.f, 0.f, 0.f};
        qmul_adj(lqs[q], ql, lqb, lqbb, qlb);
        const float thb = -sn[q] * qlb[0] + cs[q] * (jr.axis[0] * qlb[1] + jr.axis[1] * qlb[2] + jr.axis[2] * qlb[3]);
        A->qposb[jr.qadr] += 0.5f * thb;
        // anc = lp_before + mat_before jpos, ax = mat_before jaxis (+ their world-frame cotangents)
        for (int i = 0; i < 3; i++) ancb[i] += A->ftmp[j][i];
        float mb[9];
        for (int i = 0; i < 3; i++)
          for (int k = 0; k < 3; k++) mb[3 * i + k] = ancb[i] * jr.pos[k] + A->ftmp[j][3 + i] * jr.axis[k];
        q2m_adj(lqs[q], mb, lqbb);
        for (int i = 0; i < 3; i++) lpb[i] = ancb[i];
        for (int i = 0; i < 4; i++) lqb[i] = lqbb[i];
      }
    }
  }
  SYNC();
  TACC(24, tk, lane);
}

// ------------------------------------------------------------------- VJP kernel
struct VjpArgs {
  const float *act, *g_qpos, *g_qvel, *g_rew, *g_aux;  // act / g_rew / g_aux: env mode only
  float *o_qpos, *o_qvel, *o_ctrl, *o_aux;
  float* scratch;                                     // per env: row slab, then the adjoint scratch
  int scratch_stride, row_floats;
  float* nonfinite;  // optional: envs whose cotangents came out non-finite get zero outputs, counted here
  float* unr;        // unrolled mode (MJL_OPT_VJP_UNROLLED): per env tape + row accumulators, else null
  TapeDims td;
  const float* g_ws; // optional: cotangent of the output qacc_warmstart (= qacc)
  float* o_ws;       // optional: cotangent of the input qacc_warmstart (unrolled mode, warm start taken)
  // VJP tape (record / replay): this step's slot, per env `slot_stride` floats: the workspace after
  // integrate [s_w], the pre-step qpos / qvel / aux and the forward's a', factor of Hc [s_a], the
  // constraint rows [s_r], the solve tape (unrolled) [s_t]
  float* slot;
  long long slot_stride;
  int s_w, s_a, s_r, s_t;
  ApgPostArgs post;  // record: the APG post-step update fused into the launch (post.alive null: none)
  ApgNextArgs next;  // record with post: the next step's observation + policy forward (next.o null: none)
  ApgPolicyBwd pbwd; // replay (ENV): the policy + observation backward added to the state cotangents (P.nl 0: none)
};

// record mode's share of WSA: what the forward leaves there for the reverse passes
template <class DM> struct WSAR {
  static constexpr int NV = DM::NV, LD = DM::LD;
  float qpos0[MJL_MAXQ], qvel0[LD];
  alignas(16) float Lc[NV * LD];
  alignas(16) float invdc[LD];
  float ap[LD];
};
// slot layout of the A part: qpos0 [MAXQ], qvel0 [LD], aux [12], ap [LD], invdc [LD], Lc [NV * LD]
template <class DM> __host__ __device__ constexpr int slot_a_floats() {
  return MJL_MAXQ + DM::LD + 12 + 2 * DM::LD + DM::NV * DM::LD;
}
template <class DM> __host__ __device__ constexpr int slot_w_floats() { return (int)(sizeof(WS<DM>) / 4); }

// record / replay of the A part (lanes stride the arrays)
template <class DM, class AT> INL void slot_a_io(GLBA float* sa, AT* A, LDSA float* aux, int lane, bool store) {
  constexpr int LD = DM::LD, NV = DM::NV;
  auto mv = [&](LDSA float* l, GLBA float* g, int n) {
    for (int i = lane; i < n; i += 64) { if (store) g[i] = l[i]; else l[i] = g[i]; }
  };
  mv((LDSA float*)A->qpos0, sa, MJL_MAXQ);
  mv((LDSA float*)A->qvel0, sa + MJL_MAXQ, LD);
  mv(aux, sa + MJL_MAXQ + LD, MJL_AUX_DIM);
  mv((LDSA float*)A->ap, sa + MJL_MAXQ + LD + 12, LD);
  mv((LDSA float*)A->invdc, sa + MJL_MAXQ + 2 * LD + 12, LD);
  mv((LDSA float*)A->Lc, sa + MJL_MAXQ + 3 * LD + 12, NV * LD);
}

// replay's load of a tape slot into LDS: every global load of the workspace (b128) and of the A part
// issued before the first LDS store (as a loop of load -> store pairs each iteration waited for its
// own load: ~28 dependent HBM round trips per replayed step)
template <class DM, class AT> INL void slot_replay_load(GLBA const float* sw, GLBA const float* sa, LDSA WS<DM>* W,
                                                      AT* A, LDSA float* aux, int lane) {
  constexpr int LD = DM::LD, NV = DM::NV;
  constexpr int NW = (int)(sizeof(WS<DM>) / 16), QW = (NW + 63) / 64;
  constexpr int NA = slot_a_floats<DM>(), QA = (NA + 63) / 64;
  constexpr int O1 = MJL_MAXQ, O2 = O1 + LD, O3 = O2 + 12, O4 = O3 + LD, O5 = O4 + LD;  // A-part segments
  f32x4 w[QW];
  float a[QA];
#pragma unroll
  for (int q = 0; q < QW; q++) {
    const int i = lane + 64 * q;
    if (i < NW) w[q] = ((GLBA const f32x4*)sw)[i];
  }
#pragma unroll
  for (int q = 0; q < QA; q++) {
    const int i = lane + 64 * q;
    a[q] = i < NA ? sa[i] : 0.f;
  }
#pragma unroll
  for (int q = 0; q < QW; q++) {
    const int i = lane + 64 * q;
    if (i < NW) ((LDSA f32x4*)W)[i] = w[q];
  }
#pragma unroll
  for (int q = 0; q < QA; q++) {
    const int i = lane + 64 * q;
    if (i < O1) ((LDSA float*)A->qpos0)[i] = a[q];
    else if (i < O2) ((LDSA float*)A->qvel0)[i - O1] = a[q];
    else if (i < O3) { if (i - O2 < MJL_AUX_DIM) aux[i - O2] = a[q]; }
    else if (i < O4) ((LDSA float*)A->ap)[i - O3] = a[q];
    else if (i < O5) ((LDSA float*)A->invdc)[i - O4] = a[q];
    else if (i < NA) ((LDSA float*)A->Lc)[i - O5] = a[q];
  }
  (void)NV;
}

// the lean replay's slot load: the workspace image minus its matrix block (M, H, invd stay in the slot)
// into WSB, and the A part's pre-step state, aux and a' (Lc, invdc stay in the slot); all global loads
// issued before the first LDS store, as slot_replay_load (the image by LDS-DMA instead, lane-linear
// global_load_lds_dwordx4: 101.6 against 101.3 us per replay, not kept)
template <class DM> INL void slot_replay_load_lean(GLBA const float* sw, GLBA const float* sa, LDSA WSB<DM>* W,
                                                   LDSA WSAL<DM>* A, LDSA float* aux, int lane) {
  constexpr int LD = DM::LD;
  constexpr int MOFF = (int)(offsetof(WS<DM>, M) / 16), TOFF = (int)(offsetof(WS<DM>, frc_bias) / 16);
  constexpr int NB16 = (int)(sizeof(WSB<DM>) / 16), QW = (NB16 + 63) / 64;
  static_assert(offsetof(WSB<DM>, frc_bias) == offsetof(WS<DM>, M) && offsetof(WS<DM>, M) % 16 == 0 &&
                    offsetof(WS<DM>, frc_bias) % 16 == 0 &&
                    sizeof(WSB<DM>) + (offsetof(WS<DM>, frc_bias) - offsetof(WS<DM>, M)) == sizeof(WS<DM>),
                "WSB is WS without its matrix block");
  constexpr int O1 = MJL_MAXQ, O2 = O1 + LD, O3 = O2 + 12, O4 = O3 + LD;  // A-part segments up to a'
  constexpr int QA = (O4 + 63) / 64;
  f32x4 w[QW];
  float a[QA];
#pragma unroll
  for (int q = 0; q < QW; q++) {
    const int i = lane + 64 * q;  // WSB index; the slot's WS image has the matrix block at [MOFF, TOFF)
    if (i < NB16) w[q] = ((GLBA const f32x4*)sw)[i < MOFF ? i : i + (TOFF - MOFF)];
  }
#pragma unroll
  for (int q = 0; q < QA; q++) {
    const int i = lane + 64 * q;
    a[q] = i < O4 ? sa[i] : 0.f;
  }
#pragma unroll
  for (int q = 0; q < QW; q++) {
    const int i = lane + 64 * q;
    if (i < NB16) ((LDSA f32x4*)W)[i] = w[q];
  }
#pragma unroll
  for (int q = 0; q < QA; q++) {
    const int i = lane + 64 * q;
    if (i < O1) ((LDSA float*)A->qpos0)[i] = a[q];
    else if (i < O2) ((LDSA float*)A->qvel0)[i - O1] = a[q];
    else if (i < O3) { if (i - O2 < MJL_AUX_DIM) aux[i - O2] = a[q]; }
    else if (i < O4) ((LDSA float*)A->ap)[i - O3] = a[q];
  }
}

// One wave per env: recompute the step from the batch state (not modified), then run the reverse
// passes. ENV: the env step of envs.py (action flip / clip, reward, aux) without the reset merge.
// TM (VJP tape): 0 recompute, as above; 1 record: the forward only — the env step itself (outputs
// and state write-back as mjl_env_step without auto-reset) — leaving in the step's tape slot what
// the reverse passes read; 2 replay: the reverse passes from the slot, no recompute.
// LEAN (replay, implicit VJP): the forward workspace without its matrices (WSB) and the adjoint one
// without its dense arrays (WSAL) in LDS -- M, H, invd, Lc, invdc read from the tape slot, M-bar formed
// from its rank-one terms -- so the block fits 20 KB and 2048 envs run as one round of 8 per CU.
template <class D, bool ENV, int TM, bool LEAN = false>
__global__ __launch_bounds__(64, LEAN ? 2 : 1) void vjp_kernel(KParams P, VjpArgs V) {
  static_assert(!LEAN || TM == 2, "the lean layout is the replay's");
  typedef typename std::conditional<LEAN, WSAL<D>, typename std::conditional<TM == 1, WSAR<D>, WSA<D>>::type>::type AT;
  typedef typename std::conditional<LEAN, WSB<D>, WS<D>>::type WT;
  static_assert(!LEAN || sizeof(WT) + sizeof(AT) + 4 * (MJL_AUX_DIM + 3) <= kLdsBudget,
                "lean replay workspace exceeds the 8-waves-per-CU LDS budget");
  __shared__ WT Ws;
  __shared__ AT As;
  __shared__ float aux_s[MJL_AUX_DIM + 3];
  LDSA WT* W = (LDSA WT*)&Ws;
  LDSA AT* A = (LDSA AT*)&As;
  LDSA float* aux = (LDSA float*)aux_s;
  constexpr int LD = D::LD;
  MP m = (MP)P.m;
  // env = blockIdx.x: the XCD-aware order of the step kernel (block_env) measured 0.5 % slower here
  // (101.2 / 101.4 against 100.7 / 100.7 us per replay, 2048 envs) for 3.7 % less traffic
  const int env = blockIdx.x, lane = threadIdx.x;
  if (env >= P.nenv) return;
  const int nq = m->nq, nv = m->nv, nu = m->nu;
  const StateBuf& S = P.s;
  if constexpr (TM != 1) {  // the VJP is linear in the cotangents: all-zero in -> all-zero out, without
     // the recompute (envs past termination in an APG rollout; also keeps 0 * non-finite out of their outputs)
    // clamped-index loads (no branch around each): all issue before the first compare
    const int iq = lane < nq ? lane : max(nq - 1, 0), iv = lane < nv ? lane : max(nv - 1, 0);
    const int ia = lane < MJL_AUX_DIM ? lane : MJL_AUX_DIM - 1;
    const float cq = nq > 0 ? V.g_qpos[(size_t)env * nq + iq] : 0.f, cv = nv > 0 ? V.g_qvel[(size_t)env * nv + iv] : 0.f;
    const float cw = (V.g_ws && nv > 0) ? V.g_ws[(size_t)env * nv + iv] : 0.f;
    const float cr = ENV ? V.g_rew[env] : 0.f, ca = ENV ? V.g_aux[(size_t)env * MJL_AUX_DIM + ia] : 0.f;
    bool nz = (lane < nq && cq != 0.f) || (lane < nv && (cv != 0.f || cw != 0.f));
    if (ENV) nz = nz || (lane == 0 && cr != 0.f) || (lane < MJL_AUX_DIM && ca != 0.f);
    if (__ballot(nz) == 0ull) {
      if (lane < nq) V.o_qpos[(size_t)env * nq + lane] = 0.f;
      if (lane < nv) V.o_qvel[(size_t)env * nv + lane] = 0.f;
      if (lane < nu) V.o_ctrl[(size_t)env * nu + lane] = 0.f;
      if (ENV && lane < MJL_AUX_DIM) V.o_aux[(size_t)env * MJL_AUX_DIM + lane] = 0.f;
      if (V.o_ws && lane < nv) V.o_ws[(size_t)env * nv + lane] = 0.f;
      return;
    }
  }
  float* scr_env = V.scratch + (size_t)env * (size_t)V.scratch_stride;
  GLBA float* scr_adj = (GLBA float*)(scr_env + V.row_floats);
  GLBA float* slot = TM ? (GLBA float*)(V.slot + (size_t)env * (size_t)V.slot_stride) : nullptr;
  {  // zero the adjoint workspace and the LD-wide vectors of the forward one
    LDSA float* a = (LDSA float*)A;
    for (int i = lane; i < (int)(sizeof(AT) / 4); i += 64) a[i] = 0.f;
    for (int i = lane; i < LD; i += 64) {
      W->qvel[i] = 0.f; W->qacc_ws[i] = 0.f;
      W->frc_bias[i] = W->frc_passive[i] = W->frc_act[i] = W->frc_smooth[i] = W->qacc_smooth[i] = 0.f;
      W->qacc[i] = W->frc_con[i] = W->grad[i] = W->Mgrad[i] = W->search[i] = W->Ma[i] = W->Mv[i] = 0.f;
      W->gradold[i] = W->Mgradold[i] = 0.f;
    }
  }
  SYNC();
  const bool unr = V.unr != nullptr;
  SolveTape tp;
  tp.t = unr ? (TM ? slot + V.s_t : (GLBA float*)(V.unr + (size_t)env * V.td.stride)) : nullptr;
  tp.acc = unr ? (GLBA float*)(V.unr + (size_t)env * V.td.stride) + V.td.tape : nullptr;
  tp.d = V.td;
  tp.nup = tp.nls = tp.nsets = tp.overflow = 0;
  Rows<true> R = global_rows<D>(TM ? (float*)(slot + V.s_r) : scr_env, P.gmax_efc, P.gmax_con);
  if constexpr (TM == 2) {  // replay: the forward's workspace, pre-step state and factors from the slot
    STAMP(0, lane);
    if constexpr (LEAN) slot_replay_load_lean<D>(slot + V.s_w, slot + V.s_a, W, A, aux, lane);
    else slot_replay_load<D>(slot + V.s_w, slot + V.s_a, W, A, aux, lane);
    SYNC();
    STAMP(1, lane);
  } else {
  // every state load issues before the first wait (clamped lane indices, no branch per load)
  // (a zero-size field clamps to index 0 and is not read)
  const int iq = lane < nq ? lane : max(nq - 1, 0), iv = lane < nv ? lane : max(nv - 1, 0);
  const int iu = lane < nu ? lane : max(nu - 1, 0);
  const float q = nq > 0 ? S.qpos[(size_t)env * nq + iq] : 0.f;
  const float v = nv > 0 ? S.qvel[(size_t)env * nv + iv] : 0.f;
  const float w = nv > 0 ? S.qacc_warmstart[(size_t)env * nv + iv] : 0.f;
  float c = nu > 0 ? (ENV ? V.act[(size_t)env * nu + iu] : S.ctrl[(size_t)env * nu + iu]) : 0.f;
  const float t = S.time[env];
  float ax = 0.f, sgn = 1.f;
  int perm = iu;
  if (ENV) {
    const int ia = lane < MJL_AUX_DIM ? lane : MJL_AUX_DIM - 1;
    ax = S.aux[(size_t)env * MJL_AUX_DIM + ia];
    perm = nu > 0 ? P.env->act_perm[iu] : 0;
    sgn = nu > 0 ? P.env->act_sign[iu] : 1.f;
  }
  if (lane < nq) { W->qpos[lane] = q; A->qpos0[lane] = q; }
  if (lane < nv) { W->qvel[lane] = v; A->qvel0[lane] = v; W->qacc_ws[lane] = w; }
  if (lane == 0) W->sc[SC_TIME] = t;
  if (ENV) {  // flip + clip the action (envs.py:335-344): act[perm[j]] from lane perm[j]
    if (lane < MJL_AUX_DIM) aux[lane] = ax;
    const bool flip = rdlane(ax, 0) > 0.5f;
    const float ap = __shfl(c, perm);
    c = fminf(fmaxf(flip ? ap * sgn : c, -1.f), 1.f);
    if (TM == 1 && lane == 0) W->sc[SC_FLIP] = ax;
  }
  if (lane < nu) W->ctrl[lane] = c;
  SYNC();
  // ---- forward (forward() + integrate(), rows in the env's global slab)
  STAMP(0, lane);
  {
    const KinPre kp = kin_prefetch(m, lane);
    kinematics<D>(m, W, lane, kp);
    com_pos_crb<D>(m, W, lane, kp);
    velocity_stage<D>(m, W, lane, kp);
  }
  {
    const float x = chol_factor_solve<D>(W->M, W->H, W->invd, nv, W->frc_smooth, lane);
    if (lane < LD) W->qacc_smooth[lane] = (lane < nv) ? x : 0.f;
    SYNC();
  }
  if constexpr (TM == 1) {  // unrolled CG: chol(M) -- the reverse sweep's preconditioner -- in the slot's Lc
    if (unr && m->solver != MJL_SOLVER_NEWTON) {
      for (int i = lane; i < D::NV * LD; i += 64) A->Lc[i] = W->H[i];
      if (lane < LD) A->invdc[lane] = W->invd[lane];
      SYNC();
    }
  }
  build_rows<D, true>(m, W, R, lane);
  if (unr) {
    solver_t<D, true>(m, W, R, lane, tp);  // the same solve, recording its tape
    tp.finish(lane);
    SYNC();
  } else {
    solver<D, true>(m, W, R, lane);
  }
  sensors<D, true>(m, W, R, lane);
  if (!unr) {
    solver_hessian<D, true>(m, W, R, lane);  // Hc at the converged active set
    chol_factor_solve<D>(W->H, A->Lc, A->invdc, nv, W->frc_smooth, lane);
    SYNC();
  }
  integrate<D>(m, W, lane, A->ap);
  STAMP(1, lane);
  if constexpr (TM == 1) {  // record: the workspace as the reverse passes find it, then the env step
    {
      const LDSA f32x4* src = (const LDSA f32x4*)W;
      GLBA f32x4* dst = (GLBA f32x4*)(slot + V.s_w);
      for (int i = lane; i < (int)(sizeof(WS<D>) / 16); i += 64) dst[i] = src[i];
      slot_a_io<D>(slot + V.s_a, A, aux, lane, true);
    }
    float* obs = P.obs + (size_t)env * P.env->obs_dim;
    env_post<D>(m, W, P.env, aux, obs, lane, false);
    if (lane == 0) { P.rew[env] = W->sc[SC_REW]; P.term[env] = W->sc[SC_TERM]; P.trunc[env] = W->sc[SC_TRUNC]; }
    SYNC();
    if (lane < nq) S.qpos[(size_t)env * nq + lane] = W->qpos[lane];
    if (lane < nv) {
      S.qvel[(size_t)env * nv + lane] = W->qvel[lane];
      S.qacc_warmstart[(size_t)env * nv + lane] = W->qacc_ws[lane];
    }
    if (lane < nu) S.ctrl[(size_t)env * nu + lane] = W->ctrl[lane];
    if (lane == 0) S.time[env] = W->sc[SC_TIME];
    if (lane < MJL_AUX_DIM) S.aux[(size_t)env * MJL_AUX_DIM + lane] = aux[lane];
    return;
  }
  }
  if constexpr (TM != 1) {
  // ---- reverse
  const auto mats = [&] {
    if constexpr (LEAN) {
      GLBA const float* sw = slot + V.s_w;
      GLBA const float* sa = slot + V.s_a;
      constexpr int O4 = MJL_MAXQ + 2 * LD + 12, O5 = O4 + LD;  // invdc, Lc in the A part (slot_a_io)
      return AdjMats<GLBA const float*>{sw + offsetof(WS<D>, M) / 4, sw + offsetof(WS<D>, H) / 4,
                                        sw + offsetof(WS<D>, invd) / 4, sa + O5, sa + O4,
                                        (GLBA float*)(scr_adj + adj_scratch_floats(P.gmax_efc, P.gmax_con))};
    } else {
      return AdjMats<const LDSA float*>{W->M, W->H, W->invd, A->Lc, A->invdc, nullptr};
    }
  }();
  if constexpr (LEAN) {  // unrolled: zero this env's M-bar scratch rows
    if (unr && lane < nv) {
      GLBA f32x4* g = (GLBA f32x4*)(mats.Mb + lane * LD);
#pragma unroll
      for (int q = 0; q < LD / 4; q++) g[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  const float* gq = V.g_qpos + (size_t)env * nq;
  if (lane < nv) A->vtmp[lane] = V.g_qvel[(size_t)env * nv + lane];
  SYNC();
  if (ENV) adj_env<D>(m, W, A, (CP)P.env, (const float*)aux, V.g_rew[env], V.g_aux + (size_t)env * MJL_AUX_DIM, lane);
  STAMP(14, lane);
  // the dense arrays (mats): in LDS, or (lean) in the slot's workspace image and A part in global memory
  adj_integrate<D>(m, W, A, mats, gq, unr, lane);
  if (V.g_ws && lane < nv) A->qaccb[lane] += V.g_ws[(size_t)env * nv + lane];  // output warm start = qacc
  SYNC();
  STAMP(2, lane);
  if (unr) adj_solver_unrolled<D>(m, W, A, mats, R, scr_adj, P.gmax_efc, tp, lane);
  else adj_solver_rows<D>(m, W, A, mats, R, scr_adj, P.gmax_efc, lane);
  STAMP(3, lane);
  adj_contact_jac<D>(m, W, A, R, scr_adj, P.gmax_efc, unr ? (GLBA const float*)(tp.acc + 4 * P.gmax_efc) : nullptr,
                     lane);
  STAMP(4, lane);
  adj_collision<D>(m, W, A, R, scr_adj, P.gmax_efc, lane);
  STAMP(5, lane);
  adj_geom_frames<D>(m, A, lane);
  STAMP(6, lane);
  adj_forces<D>(m, W, A, lane);
  STAMP(7, lane);
  adj_rne<D>(m, W, A, lane);
  STAMP(8, lane);
  adj_mass<D>(m, W, A, mats, unr, lane);
  STAMP(9, lane);
  adj_crb<D>(m, A, lane);
  STAMP(10, lane);
  adj_cinert<D>(m, W, A, lane);
  STAMP(11, lane);
  adj_cdof<D>(m, W, A, lane);
  STAMP(12, lane);
  adj_kinematics<D>(m, W, A, lane);
  STAMP(13, lane);
  // ---- outputs
  // an unrolled solve whose tape overflowed (more line-search points or iterations than it holds;
  // mjl_batch_set_option rejects the models that can) has no valid derivative: NaN, or cut by the guard
  const bool tape_over = unr && tp.t[3] != 0.f;
  if (tape_over && !V.nonfinite) {
    const float nan = __builtin_nanf("");
    if (lane < nq) A->qposb[lane] = nan;
    if (lane < nv) { A->qvelb[lane] = nan; A->wsb[lane] = nan; }
    if (lane < nu) A->ctrlb[lane] = nan;
    if (ENV && lane < MJL_AUX_DIM) A->auxb[lane] = nan;
    SYNC();
  }
  if (V.nonfinite) {  // cut an env whose cotangents overflowed from the gradient (APG guard)
    bool bad = (lane < nq && !isfinite(A->qposb[lane])) || (lane < nv && !isfinite(A->qvelb[lane])) ||
               (lane < nu && !isfinite(A->ctrlb[lane])) || (ENV && lane < MJL_AUX_DIM && !isfinite(A->auxb[lane])) ||
               (lane < nv && !isfinite(A->wsb[lane])) || tape_over;
    if (__ballot(bad) != 0ull) {
      if (lane < nq) V.o_qpos[(size_t)env * nq + lane] = 0.f;
      if (lane < nv) V.o_qvel[(size_t)env * nv + lane] = 0.f;
      if (lane < nu) V.o_ctrl[(size_t)env * nu + lane] = 0.f;
      if (ENV && lane < MJL_AUX_DIM) V.o_aux[(size_t)env * MJL_AUX_DIM + lane] = 0.f;
      if (V.o_ws && lane < nv) V.o_ws[(size_t)env * nv + lane] = 0.f;
      if (lane == 0) atomicAdd(V.nonfinite, 1.f);
      return;
    }
  }
  // the APG policy's backward rides along (replay, ENV): the action cotangent through the policy and the
  // observation is added to the state cotangents before they are written (as mjl_apg_policy_bwd_obs_vjp
  // adds it to them after); the smooth-dynamics scratch (dead after the reverse passes) holds its rows
  const bool pol = ENV && TM == 2 && V.pbwd.P.nl > 0;
  LDSA float* gsrc = (LDSA float*)W->cinert;  // [32] action cotangent by action, [2][64] layer rows, [64] obs part
  if (lane < nu) {
    if (ENV) {  // ctrl = clip(flip ? act[perm] * sign : act, -1, 1)
      const mjlEnvConfig* c = P.env;
      const bool flip = aux[0] > 0.5f;
      const int src = flip ? c->act_perm[lane] : lane;
      const float sg = flip ? (float)c->act_sign[lane] : 1.f;
      const float a = V.act[(size_t)env * nu + src] * sg;
      const float ga = (a > -1.f && a < 1.f) ? sg * A->ctrlb[lane] : 0.f;
      V.o_ctrl[(size_t)env * nu + src] = ga;
      if (pol) gsrc[src] = ga;
    } else {
      V.o_ctrl[(size_t)env * nu + lane] = A->ctrlb[lane];
    }
  }
  float gq_add = 0.f, gv_add = 0.f;
  if (pol) {  // small_mlp_bwd_input_kernel<true>'s sums, then apg_obs_vjp_kernel's element
    const ApgPolicyBwd& Q = V.pbwd;
    static_assert((10 + 10 + 6 + 6) * D::NB >= 32 + 3 * 64, "policy backward scratch (cinert..cacc)");
    LDSA float* g = gsrc + 32;   // [2][64]
    LDSA float* ggs = g + 128;   // [64]: the observation's cotangent by input index
    const int L = Q.P.nl, NL = Q.P.n[L - 1], k0 = Q.P.k0;
    SYNC();
    if (lane < NL) {
      const float y = Q.P.y[L - 1][(size_t)env * NL + lane];
      g[lane] = gsrc[lane] * (1.f - y * y);
    }
    int cur = 0;
    for (int l = L - 1; l >= 0; l--) {
      const int N = Q.P.n[l], K = l ? Q.P.n[l - 1] : k0;
      const float* __restrict__ Wl = Q.P.w[l];
      SYNC();
      if (lane < K) {
        float sacc = 0.f;
        for (int jj = 0; jj < N; jj++) sacc = fmaf(Wl[jj * K + lane], g[cur * 64 + jj], sacc);
        if (l) {
          const float y = Q.P.y[l - 1][(size_t)env * K + lane];
          g[(cur ^ 1) * 64 + lane] = sacc * (1.f - y * y);
        } else {
          float gg = 0.f;
          if (Q.snap[env]) {
            gg = sacc;
            if (Q.use_norm) {
              const float den = sqrt_rn(Q.var[lane]) + 1e-8f;
              const float yy = div_rn(Q.o[(size_t)env * K + lane] - Q.mean[lane], den);
              gg = (yy >= -10.f && yy <= 10.f) ? div_rn(gg, den) : 0.f;
            }
          }
          ggs[lane] = gg;
        }
      }
      cur ^= 1;
    }
    SYNC();
    if (lane < nq) gq_add = ggs[lane];
    if (lane < nv) gv_add = ggs[nq + lane];
  }
  if (lane < nq) V.o_qpos[(size_t)env * nq + lane] = pol ? A->qposb[lane] + gq_add : A->qposb[lane];
  if (lane < nv) V.o_qvel[(size_t)env * nv + lane] = pol ? A->qvelb[lane] + gv_add : A->qvelb[lane];
  if (V.o_ws && lane < nv) V.o_ws[(size_t)env * nv + lane] = A->wsb[lane];
  if (ENV && lane < MJL_AUX_DIM) V.o_aux[(size_t)env * MJL_AUX_DIM + lane] = A->auxb[lane];
  }
}

// Record (implicit VJP) with the constraint rows in LDS, as mjl_env_step keeps them: rows in the
// global slab cost the record ~6 us per 2048-env launch (the same env step measured 62.1 -> 68.1 us
// with its rows forced into global memory, tools/prof_target.py apgstep). DL: the LDS workspace (the
// env step's 48 rows); DI: the dims of the tape image the replay reads (DHumV, whose union holds only
// the smooth-dynamics scratch). The slot it leaves is vjp_kernel<DI, true, 1>'s, field for field:
//  - the smooth-dynamics scratch (the image's union) goes to the slot before the rows overwrite it;
//  - the rows go to the slot's global row layout once the solve and the sensors are done;
//  - the A part has no LDS copy: qpos0 / qvel0 / aux go to the slot from registers at the start,
//    and a', the factor of Hc and its inverse diagonal are formed in the freed row area,
// so the kernel's LDS is the env step's (8 waves per CU). Rows beyond the LDS capacity take the
// global slab in the slot (record_rows_global), as vjp_kernel does for every env.
template <class DL, int MW> NOINL void record_rows_global(MP m, LDSA WS<DL>* W, float* rows, int gmax_efc, int gmax_con,
                                                          int lane) {
  Rows<true> R = global_rows<DL>(rows, gmax_efc, gmax_con);
  build_rows<DL, true>(m, W, R, lane);
  solver<DL, true>(m, W, R, lane);
  sensors<DL, true>(m, W, R, lane);
  solver_hessian<DL, true>(m, W, R, lane);  // Hc at the converged active set, into H
}

// UNR: the unrolled VJP's record (MJL_OPT_VJP_UNROLLED): the solve taped as vjp_kernel's record tapes it
// (SolveTape into slot + s_t, row accumulators in V.unr), chol(M) in the A part for CG (the reverse sweep's
// preconditioner) in place of the factor of Hc, which it does not use.
template <class DL, class DI, bool UNR = false>
__global__ __launch_bounds__(64, 2) void vjp_record_kernel(KParams P, VjpArgs V) {
  constexpr int LD = DL::LD, NV = DL::NV;
  static_assert(LD == DI::LD && NV == DI::NV, "the tape image's dims are the workspace's, rows aside");
  static_assert(offsetof(WS<DL>, cinert) == offsetof(WS<DI>, cinert) && offsetof(WS<DI>, cinert) % 16 == 0,
                "the image shares the workspace's layout up to the row / smooth-scratch union");
  static_assert(sizeof(WS<DI>) - offsetof(WS<DI>, cinert) <= sizeof(WS<DL>) - offsetof(WS<DL>, cinert),
                "the image's union is a prefix of the workspace's");
  static_assert(2 * LD + NV * LD <= DL::CAP * LD, "a', 1/diag and the Hc factor fit in the row area");
  static_assert(MJL_MAXQ <= 64 && LD <= 64 && MJL_AUX_DIM <= 12, "one lane per pre-step entry");
  static_assert(sizeof(WS<DL>) + 4 * (MJL_AUX_DIM + 3) <= kLdsBudget, "record workspace exceeds the 8-waves-per-CU LDS budget");
  __shared__ WS<DL> Ws;
  __shared__ float aux_s[MJL_AUX_DIM + 3];  // (as the env step kernel's: env_post's scratch past the aux)
  LDSA WS<DL>* W = (LDSA WS<DL>*)&Ws;
  LDSA float* aux = (LDSA float*)aux_s;
  MP m = (MP)P.m;
  const int env = blockIdx.x, lane = threadIdx.x;
  if (env >= P.nenv) return;
  const int nq = m->nq, nv = m->nv, nu = m->nu;
  const StateBuf& S = P.s;
  GLBA float* slot = (GLBA float*)(V.slot + (size_t)env * (size_t)V.slot_stride);
  GLBA float* sa = slot + V.s_a;
  constexpr int O1 = MJL_MAXQ, O2 = O1 + LD, O3 = O2 + 12;  // A part: qpos0, qvel0, aux, then a', 1/diag, Lc
  constexpr int U0 = (int)(offsetof(WS<DI>, cinert) / 16), NI = (int)(sizeof(WS<DI>) / 16);
  for (int i = lane; i < LD; i += 64) {  // the LD-wide vectors vjp_kernel zeroes
    W->qvel[i] = 0.f; W->qacc_ws[i] = 0.f;
    W->frc_bias[i] = W->frc_passive[i] = W->frc_act[i] = W->frc_smooth[i] = W->qacc_smooth[i] = 0.f;
    W->qacc[i] = W->frc_con[i] = W->grad[i] = W->Mgrad[i] = W->search[i] = W->Ma[i] = W->Mv[i] = 0.f;
    W->gradold[i] = W->Mgradold[i] = 0.f;
  }
  SYNC();
  // state loads as vjp_kernel's (clamped lane indices, every load before the first wait)
  const int iq = lane < nq ? lane : max(nq - 1, 0), iv = lane < nv ? lane : max(nv - 1, 0);
  const int iu = lane < nu ? lane : max(nu - 1, 0), ia = lane < MJL_AUX_DIM ? lane : MJL_AUX_DIM - 1;
  const float q = nq > 0 ? S.qpos[(size_t)env * nq + iq] : 0.f;
  const float v = nv > 0 ? S.qvel[(size_t)env * nv + iv] : 0.f;
  const float w = nv > 0 ? S.qacc_warmstart[(size_t)env * nv + iv] : 0.f;
  float c = nu > 0 ? V.act[(size_t)env * nu + iu] : 0.f;
  const float t = S.time[env];
  const float ax = S.aux[(size_t)env * MJL_AUX_DIM + ia];
  const int perm = nu > 0 ? P.env->act_perm[iu] : 0;
  const float sgn = nu > 0 ? P.env->act_sign[iu] : 1.f;
  if (lane < nq) W->qpos[lane] = q;
  if (lane < nv) { W->qvel[lane] = v; W->qacc_ws[lane] = w; }
  if (lane == 0) W->sc[SC_TIME] = t;
  if (lane < MJL_AUX_DIM) aux[lane] = ax;
  // the A part's pre-step state, straight from the registers (zero past nq / nv, as the zeroed A was)
  if (lane < MJL_MAXQ) sa[lane] = lane < nq ? q : 0.f;
  if (lane < LD) sa[O1 + lane] = lane < nv ? v : 0.f;
  if (lane < MJL_AUX_DIM) sa[O2 + lane] = ax;
  {  // flip + clip the action (envs.py:335-344): act[perm[j]] from lane perm[j]
    const bool flip = rdlane(ax, 0) > 0.5f;
    const float ap = __shfl(c, perm);
    c = fminf(fmaxf(flip ? ap * sgn : c, -1.f), 1.f);
    if (lane == 0) W->sc[SC_FLIP] = ax;
  }
  if (lane < nu) W->ctrl[lane] = c;
  SYNC();
  STAMP(0, lane);
  {
    const KinPre kp = kin_prefetch(m, lane);
    kinematics<DL>(m, W, lane, kp);
    com_pos_crb<DL>(m, W, lane, kp);
    velocity_stage<DL>(m, W, lane, kp);
  }
  {
    const float x = chol_factor_solve<DL>(W->M, W->H, W->invd, nv, W->frc_smooth, lane);
    if (lane < LD) W->qacc_smooth[lane] = (lane < nv) ? x : 0.f;
    SYNC();
  }
  SolveTape tp;  // (UNR)
  if constexpr (UNR) {
    tp.t = slot + V.s_t;
    tp.acc = (GLBA float*)(V.unr + (size_t)env * V.td.stride) + V.td.tape;
    tp.d = V.td;
    tp.nup = tp.nls = tp.nsets = tp.overflow = 0;
    // the A part's 1/diag and factor: chol(M) for CG (vjp_kernel's A->Lc / invdc), zero otherwise
    constexpr int O4 = O3 + LD, O5 = O4 + LD;
    const bool cg = m->solver != MJL_SOLVER_NEWTON;
    for (int i = lane; i < NV * LD; i += 64) sa[O5 + i] = cg ? W->H[i] : 0.f;
    for (int i = lane; i < LD; i += 64) sa[O4 + i] = cg ? W->invd[i] : 0.f;
  }
  GLBA f32x4* img = (GLBA f32x4*)(slot + V.s_w);
  {  // the image's union: the smooth-dynamics scratch, before the rows take its place
    const LDSA f32x4* src = (const LDSA f32x4*)W;
    for (int i = U0 + lane; i < NI; i += 64) img[i] = src[i];
  }
  float* rows = (float*)(slot + V.s_r);
  if (build_rows<DL, false>(m, W, lds_rows<DL>(W), lane)) {
    const Rows<false> R = lds_rows<DL>(W);
    if constexpr (UNR) {
      solver_t<DL, false>(m, W, R, lane, tp);  // the same solve, recording its tape
      tp.finish(lane);
      SYNC();
    } else {
      solver<DL, false>(m, W, R, lane);
    }
    sensors<DL, false>(m, W, R, lane);
    {  // the rows into the slot's global layout (what vjp_kernel's record leaves there)
      const Rows<true> G = global_rows<DL>(rows, P.gmax_efc, P.gmax_con);
      const int nefc = W->nefc, ncon = W->ncon;
      for (int i = lane; i < nefc * LD / 4; i += 64) ((GLBA f32x4*)G.J)[i] = ((const LDSA f32x4*)R.J)[i];
      for (int i = lane; i < nefc; i += 64) {
        G.D[i] = R.D[i]; G.aref[i] = R.aref[i]; G.jar[i] = R.jar[i]; G.force[i] = R.force[i];
        G.Jv[i] = R.Jv[i]; G.epos[i] = R.epos[i]; G.einvw[i] = R.einvw[i]; G.emeta[i] = R.emeta[i];
      }
      for (int i = lane; i < ncon * CONW; i += 64) G.con[i] = R.con[i];
      for (int i = lane; i < ncon; i += 64) { G.con_pair[i] = R.con_pair[i]; G.con_efc[i] = R.con_efc[i]; }
    }
    if constexpr (!UNR) solver_hessian<DL, false>(m, W, R, lane);  // Hc at the converged active set, into H
  } else if constexpr (UNR) {
    const Rows<true> R = global_rows<DL>(rows, P.gmax_efc, P.gmax_con);
    build_rows<DL, true>(m, W, R, lane);
    solver_t<DL, true>(m, W, R, lane, tp);
    tp.finish(lane);
    SYNC();
    sensors<DL, true>(m, W, R, lane);
  } else {
    record_rows_global<DL, 2>(m, W, rows, P.gmax_efc, P.gmax_con, lane);
  }
  // a', 1/diag and the factor of Hc in the row area (free now), zeroed as vjp_kernel's A part is
  // (UNR: a' only; 1/diag and the factor went to the slot above)
  constexpr int NAB = UNR ? LD : 2 * LD + NV * LD;
  LDSA float* ab = (LDSA float*)W->J;
  for (int i = lane; i < NAB; i += 64) ab[i] = 0.f;
  SYNC();
  if constexpr (!UNR) {
    chol_factor_solve<DL>(W->H, ab + 2 * LD, ab + LD, nv, W->frc_smooth, lane);
    SYNC();
  }
  integrate<DL>(m, W, lane, ab);
  STAMP(1, lane);
  SYNC();
  for (int i = lane; i < NAB; i += 64) sa[O3 + i] = ab[i];
  {  // the rest of the image: the workspace up to the union
    const LDSA f32x4* src = (const LDSA f32x4*)W;
    for (int i = lane; i < U0; i += 64) img[i] = src[i];
  }
  float* obs = P.obs + (size_t)env * P.env->obs_dim;
  env_post<DL>(m, W, P.env, aux, obs, lane, false);
  if (lane == 0) { P.rew[env] = W->sc[SC_REW]; P.term[env] = W->sc[SC_TERM]; P.trunc[env] = W->sc[SC_TRUNC]; }
  SYNC();
  if (lane < nq) S.qpos[(size_t)env * nq + lane] = W->qpos[lane];
  if (lane < nv) {
    S.qvel[(size_t)env * nv + lane] = W->qvel[lane];
    S.qacc_warmstart[(size_t)env * nv + lane] = W->qacc_ws[lane];
  }
  if (lane < nu) S.ctrl[(size_t)env * nu + lane] = W->ctrl[lane];
  if (lane == 0) S.time[env] = W->sc[SC_TIME];
  if (lane < MJL_AUX_DIM) S.aux[(size_t)env * MJL_AUX_DIM + lane] = aux[lane];
  if (V.post.alive) {  // mjl_apg_post's update of this env, on the state just written back (one launch less)
    bool fin = true;
    float vmax = 0.f;
    for (int j = lane; j < nq; j += 64) fin &= isfinite(W->qpos[j]);
    for (int j = lane; j < nv; j += 64) {
      const float v = W->qvel[j];
      fin &= isfinite(v);
      vmax = fmaxf(vmax, fabsf(v));
    }
    // (the env's scalars loaded here: loaded with the state at the start instead, they stay live across
    // the step and spill -- 80.7 against 78.2 us per record)
    const bool aln = apg_post_wave(V.post, env, lane, fin, vmax, W->sc[SC_REW], W->sc[SC_TERM], W->sc[SC_TRUNC],
                                   apg_post_load(V.post, env));
    if (V.next.o) {  // the next step's observation and policy forward from this state (one launch less)
      const ApgNextArgs& X = V.next;
      const bool al = __builtin_amdgcn_readlane((int)aln, 0) != 0;  // alive after this step's update
      const int k0 = nq + nv;
      LDSA float* h = (LDSA float*)W->J;  // [2][64]: the layer inputs (the row area is free here)
      for (int k = lane; k < k0; k += 64) {
        const float v = k < nq ? W->qpos[k] : W->qvel[k - nq];
        const size_t i = (size_t)env * k0 + k;
        X.o[i] = v;
        const float xv = al ? v : 0.f;
        const float in = X.use_norm ? clamp_keep_nan(div_rn(xv - X.mean[k], sqrt_rn(X.var[k]) + 1e-8f), 10.f) : xv;
        X.on[i] = in;
        h[k] = in;
      }
      if (lane == 0) X.snap[env] = al;
      SYNC();
      int K = k0, cur = 0;
      for (int l = 0; l < X.P.nl; l++) {
        const int N = X.P.n[l];
        const float* __restrict__ wt = X.P.w[l];  // [K, N]
        float y = 0.f;
        if (lane < N) {  // small_mlp_fwd_kernel's sum: the bias, then k in order
          float s = X.P.b[l][lane];
#pragma unroll 8
          for (int k = 0; k < K; k++) s = fmaf(wt[k * N + lane], h[cur * 64 + k], s);
          y = tanhf(s);
          X.P.y[l][(size_t)env * N + lane] = y;
          h[(cur ^ 1) * 64 + lane] = y;
        }
        SYNC();
        cur ^= 1;
        K = N;
      }
    }
  }
}

}  // namespace mjl
