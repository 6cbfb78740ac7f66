// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// Serial CPU restatement of the reference hot path, used solely as the parity checker by tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg. The product path (mujoco-mjx-lab_amd/)
// never links or calls this code.
//
// What it restates (the reference delegates the physics to the third-party package
// mujoco-mjx==3.3.6 on jax==0.7.2, pinned at reference requirements.txt:17-20,26-27; that code is
// not in /root/reference and not installed here, so it is restated from the published MuJoCo
// computation pipeline, module by module):
//   mjx.step  (called at reference src/envs.py:345, mjx_humanoid_speed_test.py:54)
//     forward: kinematics, com_pos, tendon, crb/factor_m     (upstream mjx/_src/smooth.py)
//              collision primitives                          (upstream collision_primitive.py)
//              make_constraint (limits, pyramidal contacts)  (upstream constraint.py)
//              com_vel, passive, rne, actuation              (upstream smooth.py, passive.py)
//              Newton / CG primal solver                     (upstream solver.py)
//              touch sensor                                  (upstream sensor.py)
//     integrate: Euler (+eulerdamp) / implicitfast           (upstream forward.py)
//   mjx.forward (src/envs.py:112) = the same without integration.
//
// Parity status: "parity unpinned" against MJX itself (no jax/mujoco in this container and no
// golden vectors in the reference). Pinned instead by analytic known-answer tests
// (free sphere, free fall, momentum/energy invariants) in tests/test_oracle_*.py.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <vector>

#include "../include/mjx355.h"
#include "dual.hpp"  // declared before the templates so qualified std:: math calls see the overloads

namespace oracle {

constexpr double kMinVal = 1e-15;  // mjMINVAL
constexpr double kMinImp = 0.0001; // mjMINIMP
constexpr double kMaxImp = 0.9999; // mjMAXIMP

// Diagnostics of the truncated-solve study (tests/test_solver_truncation.py, tools/solver_trace.py;
// DESIGN.md "Truncated solves"). Off by default; none changes a result unless kDiagSolverQacc is set.
enum : int {
  kDiagTrace = 1,        // per-solve / per-iteration / line-search trace on stderr
  kDiagSolverQacc = 2,   // counterfactual integrator: force = M qacc (the solver's own acceleration)
                         // instead of qfrc_smooth + qfrc_constraint (MJX forward.py euler/implicit)
  kDiagCostLog = 4,      // record the cost before and after every solver iteration in g_cost_log
};
inline int g_diag = 0;
inline std::vector<double> g_cost_log;  // per solve: NaN marker, cost at the start, after each iteration
template <class R> double dbl(const R& x) { return (double)x; }

template <class R> struct Contact {
  R dist, pos[3], frame[9];  // frame rows: normal, tangent1, tangent2
  R friction[5], solref[2], solimp[5], includemargin;
  int dim, geom1, geom2, efc_adr;
};

template <class R> struct Data {
  int nq, nv, nbody;
  std::vector<R> qpos, qvel, qacc_warmstart, ctrl;
  R time = 0;
  // position stage
  std::vector<R> xpos, xquat, xmat, xipos, xanchor, xaxis, geom_xpos, geom_xmat, site_xpos, site_xmat;
  std::vector<R> subtree_com, cinert, cdof, crb, M, L;
  std::vector<R> ten_length, ten_J;
  std::vector<Contact<R>> contact;
  // constraints
  int nefc = 0;
  std::vector<R> efc_J, efc_pos, efc_margin, efc_D, efc_aref, efc_force, efc_jar;
  std::vector<int> efc_type;  // 0 joint limit, 1 tendon limit, 2 contact frictionless, 3 contact pyramidal
  std::vector<int> efc_id;
  // velocity stage
  std::vector<R> cvel, cdof_dot, qfrc_bias, qfrc_passive, qfrc_actuator, qfrc_smooth, qacc_smooth;
  std::vector<R> qacc, qfrc_constraint, sensordata;
  int solver_niter = 0;
};

// ------------------------------------------------------------------------------------------------
// small math (MuJoCo conventions: quaternion [w x y z], spatial vectors [angular; linear],
// 3x3 matrices row-major)
// ------------------------------------------------------------------------------------------------
template <class R> inline void quat_mul(R* res, const R* a, const R* b) {
  R t[4] = {a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
            a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
            a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
            a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0]};
  for (int i = 0; i < 4; i++) res[i] = t[i];
}
template <class R> inline void quat2mat(R* m, const R* q) {
  R w = q[0], x = q[1], y = q[2], z = q[3];
  m[0] = 1 - 2 * (y * y + z * z); m[1] = 2 * (x * y - w * z); m[2] = 2 * (x * z + w * y);
  m[3] = 2 * (x * y + w * z); m[4] = 1 - 2 * (x * x + z * z); m[5] = 2 * (y * z - w * x);
  m[6] = 2 * (x * z - w * y); m[7] = 2 * (y * z + w * x); m[8] = 1 - 2 * (x * x + y * y);
}
template <class R> inline void normalize4(R* q) {
  R n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < R(kMinVal)) { q[0] = 1; q[1] = q[2] = q[3] = 0; return; }
  for (int i = 0; i < 4; i++) q[i] /= n;
}
template <class R> inline void mulmv3(R* r, const R* m, const R* v) {
  R t[3];
  for (int i = 0; i < 3; i++) t[i] = m[3 * i] * v[0] + m[3 * i + 1] * v[1] + m[3 * i + 2] * v[2];
  for (int i = 0; i < 3; i++) r[i] = t[i];
}
template <class R> inline void mulmtv3(R* r, const R* m, const R* v) {
  R t[3];
  for (int i = 0; i < 3; i++) t[i] = m[i] * v[0] + m[3 + i] * v[1] + m[6 + i] * v[2];
  for (int i = 0; i < 3; i++) r[i] = t[i];
}
template <class R> inline void mulmm3(R* r, const R* a, const R* b) {
  R t[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) t[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
  for (int i = 0; i < 9; i++) r[i] = t[i];
}
template <class R> inline void cross3(R* r, const R* a, const R* b) {
  R t[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
  r[0] = t[0]; r[1] = t[1]; r[2] = t[2];
}
template <class R> inline R dot3(const R* a, const R* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// spatial cross products (MuJoCo mju_crossMotion / mju_crossForce)
template <class R> inline void cross_motion(R* res, const R* v, const R* u) {
  R a[3], b[3], c[3];
  cross3(a, v, u);
  cross3(b, v, u + 3);
  cross3(c, v + 3, u);
  res[0] = a[0]; res[1] = a[1]; res[2] = a[2];
  res[3] = b[0] + c[0]; res[4] = b[1] + c[1]; res[5] = b[2] + c[2];
}
template <class R> inline void cross_force(R* res, const R* v, const R* f) {
  R a[3], b[3], c[3];
  cross3(a, v, f);
  cross3(b, v + 3, f + 3);
  cross3(c, v, f + 3);
  res[0] = a[0] + b[0]; res[1] = a[1] + b[1]; res[2] = a[2] + b[2];
  res[3] = c[0]; res[4] = c[1]; res[5] = c[2];
}
// cinert (10): [Ixx Iyy Izz Ixy Ixz Iyz, m*cx m*cy m*cz, m] about the com-frame origin
template <class R> inline void mul_inert_vec(R* r, const R* i, const R* v) {
  r[0] = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
  r[1] = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
  r[2] = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
  r[3] = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
  r[4] = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
  r[5] = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
}

// ------------------------------------------------------------------------------------------------
template <class R> void make_data(const mjlModelDesc& m, Data<R>& d) {
  int nq = m.nq, nv = m.nv, nb = m.nbody;
  d.nq = nq; d.nv = nv; d.nbody = nb;
  d.qpos.assign(m.qpos0, m.qpos0 + nq);
  d.qvel.assign(nv, 0); d.qacc_warmstart.assign(nv, 0); d.ctrl.assign(m.nu, 0); d.time = 0;
  d.xpos.assign(3 * nb, 0); d.xquat.assign(4 * nb, 0); d.xmat.assign(9 * nb, 0); d.xipos.assign(3 * nb, 0);
  d.xanchor.assign(3 * m.njnt, 0); d.xaxis.assign(3 * m.njnt, 0);
  d.geom_xpos.assign(3 * m.ngeom, 0); d.geom_xmat.assign(9 * m.ngeom, 0);
  d.site_xpos.assign(3 * m.nsite, 0); d.site_xmat.assign(9 * m.nsite, 0);
  d.subtree_com.assign(3 * nb, 0); d.cinert.assign(10 * nb, 0); d.crb.assign(10 * nb, 0);
  d.cdof.assign(6 * nv, 0); d.cdof_dot.assign(6 * nv, 0); d.cvel.assign(6 * nb, 0);
  d.M.assign(nv * nv, 0); d.L.assign(nv * nv, 0);
  d.ten_length.assign(m.ntendon, 0); d.ten_J.assign(m.ntendon * nv, 0);
  for (auto* v : {&d.qfrc_bias, &d.qfrc_passive, &d.qfrc_actuator, &d.qfrc_smooth, &d.qacc_smooth,
                  &d.qacc, &d.qfrc_constraint})
    v->assign(nv, 0);
  d.sensordata.assign(m.nsensordata, 0);
  d.contact.clear(); d.nefc = 0;
}

// ---- kinematics (upstream smooth.kinematics; MuJoCo mj_kinematics) ----------------------------
template <class R> void kinematics(const mjlModelDesc& m, Data<R>& d) {
  d.xpos[0] = d.xpos[1] = d.xpos[2] = 0;
  d.xquat[0] = 1; d.xquat[1] = d.xquat[2] = d.xquat[3] = 0;
  quat2mat(&d.xmat[0], &d.xquat[0]);
  for (int b = 1; b < m.nbody; b++) {
    int p = m.body_parentid[b];
    R pos[3], quat[4], mat[9];
    int ja = m.body_jntadr[b], jn = m.body_jntnum[b];
    if (jn > 0 && m.jnt_type[ja] == MJL_JNT_FREE) {
      int qa = m.jnt_qposadr[ja];
      for (int i = 0; i < 3; i++) pos[i] = d.qpos[qa + i];
      for (int i = 0; i < 4; i++) quat[i] = d.qpos[qa + 3 + i];
      normalize4(quat);
      for (int i = 0; i < 3; i++) d.xanchor[3 * ja + i] = pos[i];
      quat2mat(mat, quat);
      for (int i = 0; i < 3; i++) d.xaxis[3 * ja + i] = mat[3 * i + 2];
    } else {
      R bp[3] = {R(m.body_pos[b][0]), R(m.body_pos[b][1]), R(m.body_pos[b][2])};
      R bq[4] = {R(m.body_quat[b][0]), R(m.body_quat[b][1]), R(m.body_quat[b][2]), R(m.body_quat[b][3])};
      mulmv3(pos, &d.xmat[9 * p], bp);
      for (int i = 0; i < 3; i++) pos[i] += d.xpos[3 * p + i];
      quat_mul(quat, &d.xquat[4 * p], bq);
      for (int j = ja; j < ja + jn; j++) {
        R jp[3] = {R(m.jnt_pos[j][0]), R(m.jnt_pos[j][1]), R(m.jnt_pos[j][2])};
        R jx[3] = {R(m.jnt_axis[j][0]), R(m.jnt_axis[j][1]), R(m.jnt_axis[j][2])};
        quat2mat(mat, quat);
        R anchor[3], axis[3];
        mulmv3(anchor, mat, jp);
        for (int i = 0; i < 3; i++) anchor[i] += pos[i];
        mulmv3(axis, mat, jx);
        for (int i = 0; i < 3; i++) { d.xanchor[3 * j + i] = anchor[i]; d.xaxis[3 * j + i] = axis[i]; }
        int qa = m.jnt_qposadr[j];
        R ang = d.qpos[qa] - R(m.qpos0[qa]);
        R s = std::sin(ang / 2), c = std::cos(ang / 2);
        R ql[4] = {c, jx[0] * s, jx[1] * s, jx[2] * s};
        quat_mul(quat, quat, ql);
        quat2mat(mat, quat);
        R off[3];
        mulmv3(off, mat, jp);
        for (int i = 0; i < 3; i++) pos[i] = anchor[i] - off[i];
      }
      normalize4(quat);
      quat2mat(mat, quat);
    }
    for (int i = 0; i < 3; i++) d.xpos[3 * b + i] = pos[i];
    for (int i = 0; i < 4; i++) d.xquat[4 * b + i] = quat[i];
    for (int i = 0; i < 9; i++) d.xmat[9 * b + i] = mat[i];
  }
  for (int b = 0; b < m.nbody; b++) {
    R ip[3] = {R(m.body_ipos[b][0]), R(m.body_ipos[b][1]), R(m.body_ipos[b][2])};
    mulmv3(&d.xipos[3 * b], &d.xmat[9 * b], ip);
    for (int i = 0; i < 3; i++) d.xipos[3 * b + i] += d.xpos[3 * b + i];
  }
  for (int g = 0; g < m.ngeom; g++) {
    int b = m.geom_bodyid[g];
    R gp[3] = {R(m.geom_pos[g][0]), R(m.geom_pos[g][1]), R(m.geom_pos[g][2])};
    R gq[4] = {R(m.geom_quat[g][0]), R(m.geom_quat[g][1]), R(m.geom_quat[g][2]), R(m.geom_quat[g][3])};
    mulmv3(&d.geom_xpos[3 * g], &d.xmat[9 * b], gp);
    for (int i = 0; i < 3; i++) d.geom_xpos[3 * g + i] += d.xpos[3 * b + i];
    R gm[9];
    quat2mat(gm, gq);
    mulmm3(&d.geom_xmat[9 * g], &d.xmat[9 * b], gm);
  }
  for (int s = 0; s < m.nsite; s++) {
    int b = m.site_bodyid[s];
    R sp[3] = {R(m.site_pos[s][0]), R(m.site_pos[s][1]), R(m.site_pos[s][2])};
    R sq[4] = {R(m.site_quat[s][0]), R(m.site_quat[s][1]), R(m.site_quat[s][2]), R(m.site_quat[s][3])};
    mulmv3(&d.site_xpos[3 * s], &d.xmat[9 * b], sp);
    for (int i = 0; i < 3; i++) d.site_xpos[3 * s + i] += d.xpos[3 * b + i];
    R sm[9];
    quat2mat(sm, sq);
    mulmm3(&d.site_xmat[9 * s], &d.xmat[9 * b], sm);
  }
}

// ---- com_pos (upstream smooth.com_pos; MuJoCo mj_comPos) -------------------------------------
template <class R> void com_pos(const mjlModelDesc& m, Data<R>& d) {
  for (int b = 0; b < m.nbody; b++) {
    R ms = 0, acc[3] = {0, 0, 0};
    for (int c = b; c < m.body_subtree_end[b]; c++) {
      ms += R(m.body_mass[c]);
      for (int i = 0; i < 3; i++) acc[i] += R(m.body_mass[c]) * d.xipos[3 * c + i];
    }
    for (int i = 0; i < 3; i++) d.subtree_com[3 * b + i] = ms < R(kMinVal) ? d.xipos[3 * b + i] : acc[i] / ms;
  }
  for (int b = 0; b < m.nbody; b++) {
    R* ci = &d.cinert[10 * b];
    R mass = R(m.body_mass[b]);
    if (b == 0 || mass == 0) { for (int i = 0; i < 10; i++) ci[i] = 0; continue; }
    const double* t = m.body_inertia[b];
    R Ib[9] = {R(t[0]), R(t[3]), R(t[4]), R(t[3]), R(t[1]), R(t[5]), R(t[4]), R(t[5]), R(t[2])};
    const R* X = &d.xmat[9 * b];
    R tmp[9], Iw[9];
    mulmm3(tmp, X, Ib);
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) Iw[3 * i + j] = tmp[3 * i] * X[3 * j] + tmp[3 * i + 1] * X[3 * j + 1] + tmp[3 * i + 2] * X[3 * j + 2];
    int root = m.body_rootid[b];
    R c[3];
    for (int i = 0; i < 3; i++) c[i] = d.xipos[3 * b + i] - d.subtree_com[3 * root + i];
    R cc = dot3(c, c);
    ci[0] = Iw[0] + mass * (cc - c[0] * c[0]);
    ci[1] = Iw[4] + mass * (cc - c[1] * c[1]);
    ci[2] = Iw[8] + mass * (cc - c[2] * c[2]);
    ci[3] = Iw[1] - mass * c[0] * c[1];
    ci[4] = Iw[2] - mass * c[0] * c[2];
    ci[5] = Iw[5] - mass * c[1] * c[2];
    ci[6] = mass * c[0]; ci[7] = mass * c[1]; ci[8] = mass * c[2]; ci[9] = mass;
  }
  for (int dof = 0; dof < m.nv; dof++) {
    int j = m.dof_jntid[dof], b = m.dof_bodyid[dof];
    R* cd = &d.cdof[6 * dof];
    const R* com = &d.subtree_com[3 * m.body_rootid[b]];
    if (m.jnt_type[j] == MJL_JNT_FREE) {
      int k = dof - m.jnt_dofadr[j];
      for (int i = 0; i < 6; i++) cd[i] = 0;
      if (k < 3) { cd[3 + k] = 1; continue; }
      R ax[3] = {d.xmat[9 * b + (k - 3)], d.xmat[9 * b + 3 + (k - 3)], d.xmat[9 * b + 6 + (k - 3)]};
      R off[3];
      for (int i = 0; i < 3; i++) off[i] = com[i] - d.xanchor[3 * j + i];
      cd[0] = ax[0]; cd[1] = ax[1]; cd[2] = ax[2];
      cross3(cd + 3, ax, off);
    } else {
      const R* ax = &d.xaxis[3 * j];
      R off[3];
      for (int i = 0; i < 3; i++) off[i] = com[i] - d.xanchor[3 * j + i];
      cd[0] = ax[0]; cd[1] = ax[1]; cd[2] = ax[2];
      cross3(cd + 3, ax, off);
    }
  }
}

// ---- fixed tendons (upstream smooth.tendon) --------------------------------------------------
template <class R> void tendon(const mjlModelDesc& m, Data<R>& d) {
  for (int t = 0; t < m.ntendon; t++) {
    R len = 0;
    for (int k = 0; k < m.nv; k++) d.ten_J[t * m.nv + k] = 0;
    for (int w = 0; w < m.tendon_num[t]; w++) {
      int j = m.tendon_jnt[t][w];
      R c = R(m.tendon_coef[t][w]);
      len += c * d.qpos[m.jnt_qposadr[j]];
      d.ten_J[t * m.nv + m.jnt_dofadr[j]] += c;
    }
    d.ten_length[t] = len;
  }
}

// ---- crb + dense M (upstream smooth.crb; MuJoCo mj_crb) --------------------------------------
template <class R> void crb(const mjlModelDesc& m, Data<R>& d) {
  for (int b = 0; b < m.nbody; b++)
    for (int i = 0; i < 10; i++) {
      R s = 0;
      for (int c = b; c < m.body_subtree_end[b]; c++) s += d.cinert[10 * c + i];
      d.crb[10 * b + i] = s;
    }
  int nv = m.nv;
  std::fill(d.M.begin(), d.M.end(), R(0));
  for (int i = 0; i < nv; i++) {
    R f[6];
    mul_inert_vec(f, &d.crb[10 * m.dof_bodyid[i]], &d.cdof[6 * i]);
    for (int j = i; j >= 0; j = m.dof_parentid[j]) {
      R v = 0;
      for (int k = 0; k < 6; k++) v += d.cdof[6 * j + k] * f[k];
      d.M[i * nv + j] = v;
      d.M[j * nv + i] = v;
    }
    d.M[i * nv + i] += R(m.dof_armature[i]);
  }
}

// dense Cholesky A = L L^T (lower), returns false if not SPD
template <class R> bool cholesky(const R* A, R* L, int n) {
  for (int i = 0; i < n * n; i++) L[i] = 0;
  for (int j = 0; j < n; j++) {
    R s = A[j * n + j];
    for (int k = 0; k < j; k++) s -= L[j * n + k] * L[j * n + k];
    if (!(s > 0)) return false;
    R ljj = std::sqrt(s);
    L[j * n + j] = ljj;
    for (int i = j + 1; i < n; i++) {
      R t = A[i * n + j];
      for (int k = 0; k < j; k++) t -= L[i * n + k] * L[j * n + k];
      L[i * n + j] = t / ljj;
    }
  }
  return true;
}
template <class R> void chol_solve(const R* L, int n, R* x) {  // in place: x <- (L L^T)^-1 x
  for (int i = 0; i < n; i++) {
    R s = x[i];
    for (int k = 0; k < i; k++) s -= L[i * n + k] * x[k];
    x[i] = s / L[i * n + i];
  }
  for (int i = n - 1; i >= 0; i--) {
    R s = x[i];
    for (int k = i + 1; k < n; k++) s -= L[k * n + i] * x[k];
    x[i] = s / L[i * n + i];
  }
}

// ---- collision primitives (upstream collision_primitive.py, MJX 3.3 semantics) ----------------
template <class R> inline R normalize3(R* v) {
  R n = std::sqrt(dot3(v, v));
  R den = n + (n == 0 ? R(1e-6) : R(0));
  for (int i = 0; i < 3; i++) v[i] /= den;
  return n;
}
template <class R> void make_frame(R* frame, const R* a_in) {  // math.make_frame
  R a[3] = {a_in[0], a_in[1], a_in[2]};
  normalize3(a);
  R b[3] = {0, 0, 0};
  if (a[1] > R(-0.5) && a[1] < R(0.5)) b[1] = 1; else b[2] = 1;
  R ab = dot3(a, b);
  for (int i = 0; i < 3; i++) b[i] -= a[i] * ab;
  normalize3(b);
  R c[3];
  cross3(c, a, b);
  for (int i = 0; i < 3; i++) { frame[i] = a[i]; frame[3 + i] = b[i]; frame[6 + i] = c[i]; }
}
template <class R> void closest_segment_point(R* res, const R* a, const R* b, const R* pt) {
  R ab[3], ap[3];
  for (int i = 0; i < 3; i++) { ab[i] = b[i] - a[i]; ap[i] = pt[i] - a[i]; }
  R t = dot3(ap, ab) / (dot3(ab, ab) + R(1e-6));
  t = std::min(std::max(t, R(0)), R(1));
  for (int i = 0; i < 3; i++) res[i] = a[i] + t * ab[i];
}
template <class R> void closest_segment_segment(R* best_a, R* best_b, const R* a0, const R* a1,
                                                const R* b0, const R* b1) {
  R da[3], db[3];
  for (int i = 0; i < 3; i++) { da[i] = a1[i] - a0[i]; db[i] = b1[i] - b0[i]; }
  R len_a = normalize3(da), len_b = normalize3(db);
  R ha = len_a * R(0.5), hb = len_b * R(0.5);
  R am[3], bm[3], tr[3];
  for (int i = 0; i < 3; i++) { am[i] = a0[i] + da[i] * ha; bm[i] = b0[i] + db[i] * hb; tr[i] = am[i] - bm[i]; }
  R dadb = dot3(da, db), datr = dot3(da, tr), dbtr = dot3(db, tr);
  R denom = 1 - dadb * dadb;
  R ta0 = (-datr + dadb * dbtr) / (denom + R(1e-6));
  R tb0 = dbtr + ta0 * dadb;
  R ta = std::min(std::max(ta0, -ha), ha), tb = std::min(std::max(tb0, -hb), hb);
  for (int i = 0; i < 3; i++) { best_a[i] = am[i] + da[i] * ta; best_b[i] = bm[i] + db[i] * tb; }
  R na[3], nb[3];
  closest_segment_point(na, a0, a1, best_b);
  closest_segment_point(nb, b0, b1, best_a);
  R d1 = 0, d2 = 0;
  for (int i = 0; i < 3; i++) {
    d1 += (best_b[i] - na[i]) * (best_b[i] - na[i]);
    d2 += (best_a[i] - nb[i]) * (best_a[i] - nb[i]);
  }
  if (d1 < d2) { for (int i = 0; i < 3; i++) best_a[i] = na[i]; }
  else { for (int i = 0; i < 3; i++) best_b[i] = nb[i]; }
}
// sphere-sphere core: returns dist, writes pos and normal (pos1 -> pos2)
template <class R> R sphere_sphere(R* pos, R* n, const R* p1, R r1, const R* p2, R r2) {
  for (int i = 0; i < 3; i++) n[i] = p2[i] - p1[i];
  R dist = normalize3(n) - (r1 + r2);
  for (int i = 0; i < 3; i++) pos[i] = p1[i] + n[i] * (r1 + dist * R(0.5));
  return dist;
}

// Runs the pair's primitive, returns number of candidate contacts written to out[0..1]
// (dist, pos, frame); activity is decided by the caller.
template <class R> int collide_pair(const mjlModelDesc& m, const Data<R>& d, int p, R dist[2], R pos[2][3],
                                    R frame[2][9]) {
  int g1 = m.pair_geom1[p], g2 = m.pair_geom2[p];
  const R* x1 = &d.geom_xpos[3 * g1];
  const R* x2 = &d.geom_xpos[3 * g2];
  const R* m1 = &d.geom_xmat[9 * g1];
  const R* m2 = &d.geom_xmat[9 * g2];
  R r1 = R(m.geom_size[g1][0]), r2 = R(m.geom_size[g2][0]);
  R h1 = R(m.geom_size[g1][1]), h2 = R(m.geom_size[g2][1]);
  switch (m.pair_kind[p]) {
    case MJL_COL_PLANE_SPHERE: {
      R n[3] = {m1[2], m1[5], m1[8]};
      R diff[3] = {x2[0] - x1[0], x2[1] - x1[1], x2[2] - x1[2]};
      dist[0] = dot3(diff, n) - r2;
      for (int i = 0; i < 3; i++) pos[0][i] = x2[i] - n[i] * (r2 + R(0.5) * dist[0]);
      make_frame(frame[0], n);
      return 1;
    }
    case MJL_COL_PLANE_CAPSULE: {
      R n[3] = {m1[2], m1[5], m1[8]};
      R ax[3] = {m2[2], m2[5], m2[8]};
      R nd = dot3(n, ax);
      R b[3] = {ax[0] - n[0] * nd, ax[1] - n[1] * nd, ax[2] - n[2] * nd};
      R bn = normalize3(b);
      if (bn < R(0.5)) {
        b[0] = b[1] = b[2] = 0;
        if (n[1] > R(-0.5) && n[1] < R(0.5)) b[1] = 1; else b[2] = 1;
      }
      R c[3];
      cross3(c, n, b);
      for (int k = 0; k < 2; k++) {
        R sgn = k == 0 ? R(1) : R(-1);
        R sp[3];
        for (int i = 0; i < 3; i++) sp[i] = x2[i] + sgn * ax[i] * h2;
        R diff[3] = {sp[0] - x1[0], sp[1] - x1[1], sp[2] - x1[2]};
        dist[k] = dot3(diff, n) - r2;
        for (int i = 0; i < 3; i++) pos[k][i] = sp[i] - n[i] * (r2 + R(0.5) * dist[k]);
        for (int i = 0; i < 3; i++) { frame[k][i] = n[i]; frame[k][3 + i] = b[i]; frame[k][6 + i] = c[i]; }
      }
      return 2;
    }
    case MJL_COL_SPHERE_SPHERE: {
      R n[3];
      dist[0] = sphere_sphere(pos[0], n, x1, r1, x2, r2);
      make_frame(frame[0], n);
      return 1;
    }
    case MJL_COL_SPHERE_CAPSULE: {
      R ax[3] = {m2[2] * h2, m2[5] * h2, m2[8] * h2};
      R a[3] = {x2[0] - ax[0], x2[1] - ax[1], x2[2] - ax[2]};
      R bb[3] = {x2[0] + ax[0], x2[1] + ax[1], x2[2] + ax[2]};
      R pt[3], n[3];
      closest_segment_point(pt, a, bb, x1);
      dist[0] = sphere_sphere(pos[0], n, x1, r1, pt, r2);
      make_frame(frame[0], n);
      return 1;
    }
    case MJL_COL_CAPSULE_CAPSULE: {
      R s1[3] = {m1[2] * h1, m1[5] * h1, m1[8] * h1};
      R s2[3] = {m2[2] * h2, m2[5] * h2, m2[8] * h2};
      R a0[3], a1[3], b0[3], b1[3];
      for (int i = 0; i < 3; i++) {
        a0[i] = x1[i] - s1[i]; a1[i] = x1[i] + s1[i];
        b0[i] = x2[i] - s2[i]; b1[i] = x2[i] + s2[i];
      }
      R pa[3], pb[3], n[3];
      closest_segment_segment(pa, pb, a0, a1, b0, b1);
      dist[0] = sphere_sphere(pos[0], n, pa, r1, pb, r2);
      make_frame(frame[0], n);
      return 1;
    }
  }
  return 0;
}

template <class R> void collision(const mjlModelDesc& m, Data<R>& d) {
  d.contact.clear();
  for (int p = 0; p < m.npair; p++) {
    R dist[2], pos[2][3], frame[2][9];
    int n = collide_pair(m, d, p, dist, pos, frame);
    R includemargin = R(m.pair_margin[p] - m.pair_gap[p]);
    for (int k = 0; k < n; k++) {
      if (!(dist[k] - includemargin < 0)) continue;  // inactive (MJX: pos = dist - includemargin; active = pos < 0)
      Contact<R> c;
      c.dist = dist[k];
      for (int i = 0; i < 3; i++) c.pos[i] = pos[k][i];
      for (int i = 0; i < 9; i++) c.frame[i] = frame[k][i];
      for (int i = 0; i < 5; i++) { c.friction[i] = R(m.pair_friction[p][i]); c.solimp[i] = R(m.pair_solimp[p][i]); }
      c.solref[0] = R(m.pair_solref[p][0]); c.solref[1] = R(m.pair_solref[p][1]);
      c.includemargin = includemargin;
      c.dim = m.pair_condim[p];
      c.geom1 = m.pair_geom1[p]; c.geom2 = m.pair_geom2[p];
      c.efc_adr = -1;
      d.contact.push_back(c);
    }
  }
}

// translational/rotational Jacobian of a world point attached to body b (MuJoCo mj_jac)
template <class R> void jac_point(const mjlModelDesc& m, const Data<R>& d, int b, const R* pt, R* jacp, R* jacr) {
  int nv = m.nv;
  for (int i = 0; i < 3 * nv; i++) { jacp[i] = 0; if (jacr) jacr[i] = 0; }
  if (b <= 0) return;
  int dof = -1;
  for (int bb = b; bb > 0; bb = m.body_parentid[bb])
    if (m.body_dofnum[bb] > 0) { dof = m.body_dofadr[bb] + m.body_dofnum[bb] - 1; break; }
  const R* com = &d.subtree_com[3 * m.body_rootid[b]];
  R off[3] = {pt[0] - com[0], pt[1] - com[1], pt[2] - com[2]};
  for (; dof >= 0; dof = m.dof_parentid[dof]) {
    const R* c = &d.cdof[6 * dof];
    R cr[3];
    cross3(cr, c, off);
    for (int i = 0; i < 3; i++) {
      jacp[i * nv + dof] = c[3 + i] + cr[i];
      if (jacr) jacr[i * nv + dof] = c[i];
    }
  }
}

// impedance / reference parameters (upstream constraint._kbi; MuJoCo getimpedance + mj_makeImpedance)
template <class R> void kbi(const mjlModelDesc& m, const R* solref, const R* solimp, R pos, R& k, R& b, R& imp) {
  R timeconst = solref[0], dampratio = solref[1];
  timeconst = std::max(timeconst, R(2 * m.timestep));
  R dmin = std::min(std::max(solimp[0], R(kMinImp)), R(kMaxImp));
  R dmax = std::min(std::max(solimp[1], R(kMinImp)), R(kMaxImp));
  R width = std::max(R(kMinVal), solimp[2]);
  R mid = std::min(std::max(solimp[3], R(kMinImp)), R(kMaxImp));
  R power = std::max(R(1), solimp[4]);
  k = 1 / (dmax * dmax * timeconst * timeconst * dampratio * dampratio);
  b = 2 / (dmax * timeconst);
  if (solref[0] <= 0) k = -solref[0] / (dmax * dmax);
  if (solref[1] <= 0) b = -solref[1] / dmax;
  R x = std::abs(pos) / width;
  R y;
  if (x < mid) y = (1 / std::pow(mid, power - 1)) * std::pow(x, power);
  else y = 1 - (1 / std::pow(1 - mid, power - 1)) * std::pow(1 - x, power);
  imp = dmin + y * (dmax - dmin);
  imp = std::min(std::max(imp, dmin), dmax);
  if (x > 1) imp = dmax;
}

// ---- make_constraint (upstream constraint.py; MuJoCo mj_makeConstraint) -----------------------
template <class R> void make_constraint(const mjlModelDesc& m, Data<R>& d) {
  int nv = m.nv;
  d.efc_J.clear(); d.efc_pos.clear(); d.efc_margin.clear(); d.efc_D.clear(); d.efc_aref.clear();
  d.efc_type.clear(); d.efc_id.clear();
  std::vector<R> invw, solref, solimp;
  auto add_row = [&](const R* J, R pos, R margin, R iw, const R* sr, const R* si, int type, int id) {
    d.efc_J.insert(d.efc_J.end(), J, J + nv);
    d.efc_pos.push_back(pos); d.efc_margin.push_back(margin);
    invw.push_back(iw);
    solref.insert(solref.end(), sr, sr + 2);
    solimp.insert(solimp.end(), si, si + 5);
    d.efc_type.push_back(type); d.efc_id.push_back(id);
  };
  std::vector<R> J(nv);
  // joint limits (hinge): one row per limited joint, side chosen by the nearer limit
  for (int j = 0; j < m.njnt; j++) {
    if (!m.jnt_limited[j] || m.jnt_type[j] != MJL_JNT_HINGE) continue;
    R q = d.qpos[m.jnt_qposadr[j]];
    R dmin = q - R(m.jnt_range[j][0]), dmax = R(m.jnt_range[j][1]) - q;
    R dist = std::min(dmin, dmax), margin = R(m.jnt_margin[j]);
    if (!(dist - margin < 0)) continue;
    std::fill(J.begin(), J.end(), R(0));
    J[m.jnt_dofadr[j]] = dmin < dmax ? R(1) : R(-1);
    R sr[2] = {R(m.jnt_solref[j][0]), R(m.jnt_solref[j][1])};
    R si[5];
    for (int i = 0; i < 5; i++) si[i] = R(m.jnt_solimp[j][i]);
    add_row(J.data(), dist, margin, R(m.dof_invweight0[m.jnt_dofadr[j]]), sr, si, 0, j);
  }
  // tendon limits
  for (int t = 0; t < m.ntendon; t++) {
    if (!m.tendon_limited[t]) continue;
    R len = d.ten_length[t];
    R dmin = len - R(m.tendon_range[t][0]), dmax = R(m.tendon_range[t][1]) - len;
    R dist = std::min(dmin, dmax), margin = R(m.tendon_margin[t]);
    if (!(dist - margin < 0)) continue;
    R s = dmin < dmax ? R(1) : R(-1);
    for (int k = 0; k < nv; k++) J[k] = s * d.ten_J[t * nv + k];
    R sr[2] = {R(m.tendon_solref[t][0]), R(m.tendon_solref[t][1])};
    R si[5];
    for (int i = 0; i < 5; i++) si[i] = R(m.tendon_solimp[t][i]);
    add_row(J.data(), dist, margin, R(m.tendon_invweight0[t]), sr, si, 1, t);
  }
  // contacts
  std::vector<R> jp1(3 * nv), jp2(3 * nv), jd(3 * nv);
  for (size_t ci = 0; ci < d.contact.size(); ci++) {
    Contact<R>& c = d.contact[ci];
    int b1 = m.geom_bodyid[c.geom1], b2 = m.geom_bodyid[c.geom2];
    jac_point(m, d, b1, c.pos, jp1.data(), (R*)nullptr);
    jac_point(m, d, b2, c.pos, jp2.data(), (R*)nullptr);
    for (int i = 0; i < 3 * nv; i++) jd[i] = jp2[i] - jp1[i];
    R tran = R(m.body_invweight0[b1][0] + m.body_invweight0[b2][0]);
    c.efc_adr = (int)d.efc_pos.size();
    std::vector<R> Jn(nv), Jt(nv);
    for (int k = 0; k < nv; k++) Jn[k] = c.frame[0] * jd[k] + c.frame[1] * jd[nv + k] + c.frame[2] * jd[2 * nv + k];
    if (c.dim == 1) {
      add_row(Jn.data(), c.dist, c.includemargin, tran, c.solref, c.solimp, 2, (int)ci);
    } else {
      R mu = c.friction[0];
      R iw = tran + mu * mu * tran;
      iw = iw * 2 * mu * mu / R(m.impratio);
      for (int t = 1; t < c.dim; t++) {
        R mut = c.friction[t - 1];
        for (int k = 0; k < nv; k++)
          Jt[k] = c.frame[3 * t] * jd[k] + c.frame[3 * t + 1] * jd[nv + k] + c.frame[3 * t + 2] * jd[2 * nv + k];
        for (int s = 0; s < 2; s++) {
          R sg = s == 0 ? R(1) : R(-1);
          for (int k = 0; k < nv; k++) J[k] = Jn[k] + sg * mut * Jt[k];
          add_row(J.data(), c.dist, c.includemargin, iw, c.solref, c.solimp, 3, (int)ci);
        }
      }
    }
  }
  int nefc = (int)d.efc_pos.size();
  d.nefc = nefc;
  d.efc_D.resize(nefc); d.efc_aref.resize(nefc); d.efc_force.assign(nefc, 0); d.efc_jar.assign(nefc, 0);
  for (int i = 0; i < nefc; i++) {
    R k, b, imp;
    R pos = d.efc_pos[i] - d.efc_margin[i];
    kbi(m, &solref[2 * i], &solimp[5 * i], pos, k, b, imp);
    R r = std::max(invw[i] * (1 - imp) / imp, R(kMinVal));
    d.efc_D[i] = 1 / r;
    R vel = 0;
    for (int kk = 0; kk < nv; kk++) vel += d.efc_J[i * nv + kk] * d.qvel[kk];
    d.efc_aref[i] = -b * vel - k * imp * pos;
  }
}

// ---- velocity stage: com_vel, passive, rne (upstream smooth.com_vel/rne, passive.passive) ------
template <class R> void com_vel(const mjlModelDesc& m, Data<R>& d) {
  for (int i = 0; i < 6; i++) d.cvel[i] = 0;
  for (int b = 1; b < m.nbody; b++) {
    R cv[6];
    int p = m.body_parentid[b];
    for (int i = 0; i < 6; i++) cv[i] = d.cvel[6 * p + i];
    int ja = m.body_jntadr[b], jn = m.body_jntnum[b];
    for (int j = ja; j < ja + jn; j++) {
      int da = m.jnt_dofadr[j];
      if (m.jnt_type[j] == MJL_JNT_FREE) {
        for (int k = 0; k < 3; k++)
          for (int i = 0; i < 6; i++) d.cdof_dot[6 * (da + k) + i] = 0;
        for (int k = 0; k < 3; k++)
          for (int i = 0; i < 6; i++) cv[i] += d.cdof[6 * (da + k) + i] * d.qvel[da + k];
        for (int k = 3; k < 6; k++) cross_motion(&d.cdof_dot[6 * (da + k)], cv, &d.cdof[6 * (da + k)]);
        for (int k = 3; k < 6; k++)
          for (int i = 0; i < 6; i++) cv[i] += d.cdof[6 * (da + k) + i] * d.qvel[da + k];
      } else {
        cross_motion(&d.cdof_dot[6 * da], cv, &d.cdof[6 * da]);
        for (int i = 0; i < 6; i++) cv[i] += d.cdof[6 * da + i] * d.qvel[da];
      }
    }
    for (int i = 0; i < 6; i++) d.cvel[6 * b + i] = cv[i];
  }
}

template <class R> void passive(const mjlModelDesc& m, Data<R>& d) {
  for (int k = 0; k < m.nv; k++) d.qfrc_passive[k] = -R(m.dof_damping[k]) * d.qvel[k];
  for (int j = 0; j < m.njnt; j++) {
    if (m.jnt_type[j] != MJL_JNT_HINGE) continue;
    int qa = m.jnt_qposadr[j], da = m.jnt_dofadr[j];
    d.qfrc_passive[da] -= R(m.jnt_stiffness[j]) * (d.qpos[qa] - R(m.qpos_spring[qa]));
  }
}

template <class R> void rne(const mjlModelDesc& m, Data<R>& d) {
  std::vector<R> cacc(6 * m.nbody), cfrc(6 * m.nbody);
  for (int i = 0; i < 6; i++) cacc[i] = 0;
  for (int i = 0; i < 3; i++) cacc[3 + i] = -R(m.gravity[i]);
  for (int b = 1; b < m.nbody; b++) {
    int p = m.body_parentid[b];
    for (int i = 0; i < 6; i++) cacc[6 * b + i] = cacc[6 * p + i];
    for (int k = m.body_dofadr[b]; k < m.body_dofadr[b] + m.body_dofnum[b]; k++)
      for (int i = 0; i < 6; i++) cacc[6 * b + i] += d.cdof_dot[6 * k + i] * d.qvel[k];
    R f1[6], iv[6], f2[6];
    mul_inert_vec(f1, &d.cinert[10 * b], &cacc[6 * b]);
    mul_inert_vec(iv, &d.cinert[10 * b], &d.cvel[6 * b]);
    cross_force(f2, &d.cvel[6 * b], iv);
    for (int i = 0; i < 6; i++) cfrc[6 * b + i] = f1[i] + f2[i];
  }
  for (int i = 0; i < 6; i++) cfrc[i] = 0;
  for (int b = m.nbody - 1; b > 0; b--) {
    int p = m.body_parentid[b];
    if (p > 0)
      for (int i = 0; i < 6; i++) cfrc[6 * p + i] += cfrc[6 * b + i];
  }
  for (int k = 0; k < m.nv; k++) {
    R s = 0;
    for (int i = 0; i < 6; i++) s += d.cdof[6 * k + i] * cfrc[6 * m.dof_bodyid[k] + i];
    d.qfrc_bias[k] = s;
  }
}

template <class R> void actuation(const mjlModelDesc& m, Data<R>& d) {
  std::fill(d.qfrc_actuator.begin(), d.qfrc_actuator.end(), R(0));
  for (int u = 0; u < m.nu; u++) {
    R c = d.ctrl[u];
    if (m.actuator_ctrllimited[u])
      c = std::min(std::max(c, R(m.actuator_ctrlrange[u][0])), R(m.actuator_ctrlrange[u][1]));
    d.qfrc_actuator[m.jnt_dofadr[m.actuator_trnid[u]]] += R(m.actuator_gear[u]) * c;
  }
}

// ---- primal solver (upstream solver.py; MuJoCo engine_solver.c mj_solNewton / mj_solCG) --------
template <class R> struct Solver {
  const mjlModelDesc& m;
  Data<R>& d;
  int nv, nefc;
  std::vector<R> Ma, jar, grad, Mgrad, search, Mv, Jv, H, HL, gradold, Mgradold;
  R cost = 0, gauss = 0;

  Solver(const mjlModelDesc& m_, Data<R>& d_) : m(m_), d(d_), nv(m_.nv), nefc(d_.nefc) {}

  void mulM(const R* v, R* out) {
    for (int i = 0; i < nv; i++) {
      R s = 0;
      for (int k = 0; k < nv; k++) s += d.M[i * nv + k] * v[k];
      out[i] = s;
    }
  }
  R eval_cost(const R* qacc) {  // full cost at qacc (warm-start comparison)
    std::vector<R> ma(nv);
    mulM(qacc, ma.data());
    R g = 0;
    for (int i = 0; i < nv; i++) g += R(0.5) * (ma[i] - d.qfrc_smooth[i]) * (qacc[i] - d.qacc_smooth[i]);
    R c = 0;
    for (int r = 0; r < nefc; r++) {
      R j = -d.efc_aref[r];
      for (int k = 0; k < nv; k++) j += d.efc_J[r * nv + k] * qacc[k];
      if (j < 0) c += R(0.5) * d.efc_D[r] * j * j;
    }
    return g + c;
  }
  // constraint forces, cost, qfrc_constraint and gradient at the current qacc/Ma/jar
  void update() {
    R c = 0;
    for (int r = 0; r < nefc; r++) {
      R j = jar[r];
      if (j < 0) { d.efc_force[r] = -d.efc_D[r] * j; c += R(0.5) * d.efc_D[r] * j * j; }
      else d.efc_force[r] = 0;
    }
    for (int k = 0; k < nv; k++) {
      R s = 0;
      for (int r = 0; r < nefc; r++) s += d.efc_J[r * nv + k] * d.efc_force[r];
      d.qfrc_constraint[k] = s;
    }
    gauss = 0;
    for (int i = 0; i < nv; i++) gauss += R(0.5) * (Ma[i] - d.qfrc_smooth[i]) * (d.qacc[i] - d.qacc_smooth[i]);
    cost = gauss + c;
    for (int i = 0; i < nv; i++) grad[i] = Ma[i] - d.qfrc_smooth[i] - d.qfrc_constraint[i];
  }
  int nactive() const { int n = 0; for (int r = 0; r < nefc; r++) n += jar[r] < 0; return n; }
  void newton_direction() {  // Mgrad = H^-1 grad, H = M + J' D_active J
    for (int i = 0; i < nv * nv; i++) H[i] = d.M[i];
    for (int r = 0; r < nefc; r++) {
      if (!(jar[r] < 0)) continue;
      const R* J = &d.efc_J[r * nv];
      R D = d.efc_D[r];
      for (int i = 0; i < nv; i++) {
        if (J[i] == 0) continue;
        for (int k = 0; k <= i; k++) H[i * nv + k] += D * J[i] * J[k];
      }
    }
    for (int i = 0; i < nv; i++)
      for (int k = i + 1; k < nv; k++) H[i * nv + k] = H[k * nv + i];
    cholesky(H.data(), HL.data(), nv);
    for (int i = 0; i < nv; i++) Mgrad[i] = grad[i];
    chol_solve(HL.data(), nv, Mgrad.data());
  }
  void cg_precondition() {  // Mgrad = M^-1 grad
    for (int i = 0; i < nv; i++) Mgrad[i] = grad[i];
    chol_solve(d.L.data(), nv, Mgrad.data());
  }
  // cost, f'(alpha) and f''(alpha) along the search direction (MJX solver.py _LSPoint.create:
  // quad_gauss + the rows active at alpha; f'' gets mjMINVAL when the quadratic term is exactly 0)
  struct LSPoint { R alpha, cost, d0, d1; };
  LSPoint ls_point(R alpha, R gauss0, R c1, R c2) {
    R q0 = gauss0, q1 = c1, q2 = R(0.5) * c2;
    for (int r = 0; r < nefc; r++) {
      R j = jar[r] + alpha * Jv[r];
      if (j < 0) {
        R D = d.efc_D[r];
        q0 += R(0.5) * D * jar[r] * jar[r]; q1 += D * Jv[r] * jar[r]; q2 += R(0.5) * D * Jv[r] * Jv[r];
      }
    }
    LSPoint p;
    p.alpha = alpha;
    p.cost = alpha * alpha * q2 + alpha * q1 + q0;
    p.d0 = 2 * alpha * q2 + q1;
    p.d1 = 2 * q2 + (q2 == 0 ? R(kMinVal) : R(0));
    return p;
  }
  // MJX's zoom line search (mujoco-mjx 3.3.6 solver.py _linesearch): a bracket [lo, hi] around the
  // root of f', each iteration trying the Newton steps from lo and from hi and the midpoint, until
  // no bracket end moves, an end's |f'| < gtol, or ls_iterations; then the lower-cost end, taken
  // only if it improves on alpha = 0. Returns that alpha (0 = no improvement).
  R linesearch(R scale) {
    R snorm = 0;
    for (int i = 0; i < nv; i++) snorm += search[i] * search[i];
    snorm = std::sqrt(snorm);
    R gtol = R(m.tolerance * m.ls_tolerance) * snorm / scale;
    mulM(search.data(), Mv.data());
    for (int r = 0; r < nefc; r++) {
      R s = 0;
      for (int k = 0; k < nv; k++) s += d.efc_J[r * nv + k] * search[k];
      Jv[r] = s;
    }
    R c1 = 0, c2 = 0;
    for (int i = 0; i < nv; i++) { c1 += search[i] * (Ma[i] - d.qfrc_smooth[i]); c2 += search[i] * Mv[i]; }
    LSPoint p0 = ls_point(R(0), gauss, c1, c2);
    LSPoint lo = ls_point(p0.alpha - p0.d0 / p0.d1, gauss, c1, c2), hi;
    if (lo.d0 < p0.d0) hi = p0; else { hi = lo; lo = p0; }
    bool swap = true;
    for (int it = 0; it < m.ls_iterations; it++) {
      if (!swap) break;
      if (lo.d0 < 0 && lo.d0 > -gtol) break;
      if (hi.d0 > 0 && hi.d0 < gtol) break;
      LSPoint lo_next = ls_point(lo.alpha - lo.d0 / lo.d1, gauss, c1, c2);
      LSPoint hi_next = ls_point(hi.alpha - hi.d0 / hi.d1, gauss, c1, c2);
      LSPoint mid = ls_point(R(0.5) * (lo.alpha + hi.alpha), gauss, c1, c2);
      bool s1 = lo.d0 > 0 || lo.d0 < lo_next.d0;
      if (s1) lo = lo_next;
      bool s2 = mid.d0 < 0 && lo.d0 < mid.d0;
      if (s2) lo = mid;
      bool s3 = hi.d0 < 0 || hi.d0 > hi_next.d0;
      if (s3) hi = hi_next;
      bool s4 = mid.d0 > 0 && hi.d0 > mid.d0;
      if (s4) hi = mid;
      swap = s1 || s2 || s3 || s4;
    }
    bool improved = lo.cost < p0.cost || hi.cost < p0.cost;
    R alpha = lo.cost < hi.cost ? lo.alpha : hi.alpha;
    if (g_diag & kDiagTrace) {  // the zoom's result beside a brute-force scan of alpha in (0, 4]
      R best = 0, bc = p0.cost;
      for (int k = 1; k <= 4000; k++) {
        LSPoint p = ls_point(R(k) * R(0.001), gauss, c1, c2);
        if (p.cost < bc) { bc = p.cost; best = p.alpha; }
      }
      fprintf(stderr, "   ls: f(0) %.6g f'(0) %.4g | lo a %.4g f %.6g f' %.4g | hi a %.4g f %.6g f' %.4g | scan a %.4g f %.6g\n",
              dbl(p0.cost), dbl(p0.d0), dbl(lo.alpha), dbl(lo.cost), dbl(lo.d0), dbl(hi.alpha), dbl(hi.cost),
              dbl(hi.d0), dbl(best), dbl(bc));
    }
    return improved ? alpha : R(0);
  }

  void run() {
    nefc = d.nefc;
    Ma.assign(nv, 0); jar.assign(nefc, 0); grad.assign(nv, 0); Mgrad.assign(nv, 0); search.assign(nv, 0);
    Mv.assign(nv, 0); Jv.assign(nefc, 0); H.assign(nv * nv, 0); HL.assign(nv * nv, 0);
    d.solver_niter = 0;
    if (nefc == 0) {
      d.qacc = d.qacc_smooth;
      std::fill(d.qfrc_constraint.begin(), d.qfrc_constraint.end(), R(0));
      return;
    }
    R scale = R(1) / R(m.meaninertia * std::max(1, nv));
    // warm start: keep whichever of qacc_warmstart / qacc_smooth has the lower total cost
    R cw = eval_cost(d.qacc_warmstart.data());
    R cs = eval_cost(d.qacc_smooth.data());
    d.qacc = cw < cs ? d.qacc_warmstart : d.qacc_smooth;
    mulM(d.qacc.data(), Ma.data());
    for (int r = 0; r < nefc; r++) {
      R s = -d.efc_aref[r];
      for (int k = 0; k < nv; k++) s += d.efc_J[r * nv + k] * d.qacc[k];
      jar[r] = s;
    }
    update();
    if (g_diag & kDiagTrace)
      fprintf(stderr, " solve nefc %d warm start from %s (cost %.6g vs %.6g) active %d\n", nefc,
              cw < cs ? "qacc_warmstart" : "qacc_smooth", dbl(cw), dbl(cs), nactive());
    if (g_diag & kDiagCostLog) {
      g_cost_log.push_back(std::numeric_limits<double>::quiet_NaN());
      g_cost_log.push_back(dbl(cost));
    }
    bool newton = m.solver == MJL_SOLVER_NEWTON;
    if (newton) newton_direction(); else cg_precondition();
    for (int i = 0; i < nv; i++) search[i] = -Mgrad[i];
    // MJX solve(): while_loop(cond, body) with cond = niter < iterations && improvement >= tol &&
    // |grad| >= tol (improvement = inf before the first body); iterations == 1 runs body once.
    int iter = 0;
    R gnorm0 = 0;
    for (int i = 0; i < nv; i++) gnorm0 += grad[i] * grad[i];
    bool go = m.iterations == 1 || (m.iterations > 0 && scale * std::sqrt(gnorm0) >= R(m.tolerance));
    while (go) {
      R alpha = linesearch(scale);
      for (int i = 0; i < nv; i++) { d.qacc[i] += alpha * search[i]; Ma[i] += alpha * Mv[i]; }
      for (int r = 0; r < nefc; r++) jar[r] += alpha * Jv[r];
      R oldcost = cost;
      gradold = grad; Mgradold = Mgrad;
      update();
      if (newton) newton_direction(); else cg_precondition();
      iter++;
      if (newton) {
        for (int i = 0; i < nv; i++) search[i] = -Mgrad[i];
      } else {  // Polak-Ribiere, denominator floored at mjMINVAL
        R num = 0, den = 0;
        for (int i = 0; i < nv; i++) { num += grad[i] * (Mgrad[i] - Mgradold[i]); den += gradold[i] * Mgradold[i]; }
        R beta = std::max(R(0), num / std::max(R(kMinVal), den));
        for (int i = 0; i < nv; i++) search[i] = -Mgrad[i] + beta * search[i];
      }
      R improvement = scale * (oldcost - cost);
      R gnorm = 0;
      for (int i = 0; i < nv; i++) gnorm += grad[i] * grad[i];
      gnorm = scale * std::sqrt(gnorm);
      if (g_diag & kDiagCostLog) g_cost_log.push_back(dbl(cost));
      if (g_diag & kDiagTrace)
        fprintf(stderr, "  iteration %d alpha %.4g cost %.6g -> %.6g scaled |grad| %.4g active %d\n", iter,
                dbl(alpha), dbl(oldcost), dbl(cost), dbl(gnorm), nactive());
      go = m.iterations != 1 && iter < m.iterations && improvement >= R(m.tolerance) && gnorm >= R(m.tolerance);
    }
    d.solver_niter = iter;
    for (int r = 0; r < nefc; r++) d.efc_jar[r] = jar[r];
  }
};

// ---- touch sensor (upstream sensor.py; MuJoCo engine_sensor.c mjSENS_TOUCH) -------------------
template <class R> R ray_box(const R* pos, const R* mat, const double* size, const R* pnt, const R* vec) {
  R dp[3] = {pnt[0] - pos[0], pnt[1] - pos[1], pnt[2] - pos[2]};
  R lp[3], lv[3];
  mulmtv3(lp, mat, dp);
  mulmtv3(lv, mat, vec);
  R best = -1;
  for (int i = 0; i < 3; i++) {
    if (std::abs(lv[i]) <= R(kMinVal)) continue;
    for (int side = -1; side <= 1; side += 2) {
      R sol = (R(side) * R(size[i]) - lp[i]) / lv[i];
      if (sol < 0) continue;
      int i1 = (i + 1) % 3, i2 = (i + 2) % 3;
      R a = lp[i1] + sol * lv[i1], b = lp[i2] + sol * lv[i2];
      if (std::abs(a) <= R(size[i1]) && std::abs(b) <= R(size[i2]))
        if (best < 0 || sol < best) best = sol;
    }
  }
  return best;
}

template <class R> void sensors(const mjlModelDesc& m, Data<R>& d) {
  for (int s = 0; s < m.nsensor; s++) {
    R val = 0;
    int site = m.sensor_objid[s], body = m.site_bodyid[site];
    for (size_t ci = 0; ci < d.contact.size(); ci++) {
      const Contact<R>& c = d.contact[ci];
      int cb1 = m.geom_bodyid[c.geom1], cb2 = m.geom_bodyid[c.geom2];
      if (cb1 != body && cb2 != body) continue;
      R fn = 0;
      int nrow = c.dim == 1 ? 1 : 2 * (c.dim - 1);
      for (int r = 0; r < nrow; r++) fn += d.efc_force[c.efc_adr + r];
      if (fn <= 0) continue;
      R dir[3] = {c.frame[0], c.frame[1], c.frame[2]};
      if (cb2 == body) for (int i = 0; i < 3; i++) dir[i] = -dir[i];
      if (ray_box(&d.site_xpos[3 * site], &d.site_xmat[9 * site], m.site_size[site], c.pos, dir) >= 0) val += fn;
    }
    d.sensordata[m.sensor_adr[s]] = val;
  }
}

// ---- forward / integrate ----------------------------------------------------------------------
template <class R> void forward(const mjlModelDesc& m, Data<R>& d) {
  kinematics(m, d);
  com_pos(m, d);
  tendon(m, d);
  crb(m, d);
  cholesky(d.M.data(), d.L.data(), m.nv);
  collision(m, d);
  com_vel(m, d);
  make_constraint(m, d);
  passive(m, d);
  rne(m, d);
  actuation(m, d);
  for (int k = 0; k < m.nv; k++) d.qfrc_smooth[k] = d.qfrc_passive[k] - d.qfrc_bias[k] + d.qfrc_actuator[k];
  d.qacc_smooth = d.qfrc_smooth;
  chol_solve(d.L.data(), m.nv, d.qacc_smooth.data());
  Solver<R> s(m, d);
  s.run();
  // the solution seeds the next solve (MuJoCo mj_fwdConstraint; MJX solver.solve returns
  // qacc_warmstart = qacc), so it is part of forward, not of the integrator
  d.qacc_warmstart = d.qacc;
  sensors(m, d);
}

template <class R> void integrate(const mjlModelDesc& m, Data<R>& d) {
  int nv = m.nv;
  std::vector<R> qacc = d.qacc;
  bool damp = m.integrator == MJL_INT_IMPLICITFAST || m.eulerdamp;
  bool any = false;
  for (int k = 0; k < nv; k++) any |= m.dof_damping[k] > 0;
  if (damp && any) {
    std::vector<R> MI(d.M), L(nv * nv);
    for (int k = 0; k < nv; k++) MI[k * nv + k] += R(m.timestep) * R(m.dof_damping[k]);
    cholesky(MI.data(), L.data(), nv);
    for (int k = 0; k < nv; k++) qacc[k] = d.qfrc_smooth[k] + d.qfrc_constraint[k];
    if (g_diag & kDiagSolverQacc)
      for (int k = 0; k < nv; k++) {
        R s = 0;
        for (int i = 0; i < nv; i++) s += d.M[k * nv + i] * d.qacc[i];
        qacc[k] = s;
      }
    chol_solve(L.data(), nv, qacc.data());
    if (g_diag & kDiagTrace) {
      double a = 0, b = 0, c = 0;
      for (int k = 0; k < nv; k++) {
        a = std::max(a, std::abs(dbl(d.qacc[k])));
        b = std::max(b, std::abs(dbl(qacc[k])));
        c = std::max(c, std::abs(dbl(d.qfrc_constraint[k])));
      }
      fprintf(stderr, " integrate: max|qacc| solver %.4g integrator %.4g, max|qfrc_constraint| %.4g\n", a, b, c);
    }
  }
  R dt = R(m.timestep);
  for (int k = 0; k < nv; k++) d.qvel[k] += dt * qacc[k];
  for (int j = 0; j < m.njnt; j++) {
    int qa = m.jnt_qposadr[j], da = m.jnt_dofadr[j];
    if (m.jnt_type[j] == MJL_JNT_FREE) {
      for (int i = 0; i < 3; i++) d.qpos[qa + i] += dt * d.qvel[da + i];
      R w[3] = {d.qvel[da + 3], d.qvel[da + 4], d.qvel[da + 5]};
      R nrm = normalize3(w);
      R ang = nrm * dt;
      R s = std::sin(ang / 2), c = std::cos(ang / 2);
      R qr[4] = {c, w[0] * s, w[1] * s, w[2] * s};
      R* q = &d.qpos[qa + 3];
      quat_mul(q, q, qr);
      normalize4(q);
    } else {
      d.qpos[qa] += dt * d.qvel[da];
    }
  }
  d.time += dt;
}

template <class R> void step(const mjlModelDesc& m, Data<R>& d) {
  forward(m, d);
  integrate(m, d);
}

}  // namespace oracle
