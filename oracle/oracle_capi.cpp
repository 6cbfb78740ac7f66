// ORACLE — TEST INFRASTRUCTURE ONLY (see physics.hpp header). C entry points for ctypes.
#include <cstdint>

#include "env.hpp"

extern "C" {

#define ORC_MAXCON 512
#define ORC_MAXEFC 2048

typedef struct orcState {
  double qpos[MJL_MAXQ], qvel[MJL_MAXV], qacc_warmstart[MJL_MAXV], ctrl[MJL_MAXU], time;
  double qacc[MJL_MAXV], qacc_smooth[MJL_MAXV], qfrc_bias[MJL_MAXV], qfrc_passive[MJL_MAXV];
  double qfrc_actuator[MJL_MAXV], qfrc_constraint[MJL_MAXV];
  double xpos[MJL_MAXBODY][3], xquat[MJL_MAXBODY][4], xipos[MJL_MAXBODY][3], subtree_com[MJL_MAXBODY][3];
  double cvel[MJL_MAXBODY][6], cinert[MJL_MAXBODY][10], cdof[MJL_MAXV][6];
  double M[MJL_MAXV][MJL_MAXV];
  double sensordata[MJL_MAXSENSOR];
  int32_t ncon, nefc, niter, pad;
  double con_dist[ORC_MAXCON], con_pos[ORC_MAXCON][3], con_frame[ORC_MAXCON][9];
  int32_t con_geom[ORC_MAXCON][2];
  double efc_force[ORC_MAXEFC], efc_D[ORC_MAXEFC], efc_aref[ORC_MAXEFC], efc_pos[ORC_MAXEFC];
  int32_t efc_type[ORC_MAXEFC];
} orcState;

int orc_version(void) { return 1; }
int orc_state_size(void) { return (int)sizeof(orcState); }
int orc_desc_size(void) { return (int)sizeof(mjlModelDesc); }
int orc_envcfg_size(void) { return (int)sizeof(mjlEnvConfig); }

}  // extern "C"

namespace {

template <class R> void load(const mjlModelDesc& m, const orcState& s, oracle::Data<R>& d) {
  oracle::make_data(m, d);
  for (int i = 0; i < m.nq; i++) d.qpos[i] = R(s.qpos[i]);
  for (int i = 0; i < m.nv; i++) { d.qvel[i] = R(s.qvel[i]); d.qacc_warmstart[i] = R(s.qacc_warmstart[i]); }
  for (int i = 0; i < m.nu; i++) d.ctrl[i] = R(s.ctrl[i]);
  d.time = R(s.time);
}

template <class R> void save(const mjlModelDesc& m, const oracle::Data<R>& d, orcState& s) {
  int nv = m.nv;
  for (int i = 0; i < m.nq; i++) s.qpos[i] = double(d.qpos[i]);
  for (int i = 0; i < nv; i++) {
    s.qvel[i] = d.qvel[i]; s.qacc_warmstart[i] = d.qacc_warmstart[i]; s.qacc[i] = d.qacc[i];
    s.qacc_smooth[i] = d.qacc_smooth[i]; s.qfrc_bias[i] = d.qfrc_bias[i]; s.qfrc_passive[i] = d.qfrc_passive[i];
    s.qfrc_actuator[i] = d.qfrc_actuator[i]; s.qfrc_constraint[i] = d.qfrc_constraint[i];
    for (int k = 0; k < 6; k++) s.cdof[i][k] = d.cdof[6 * i + k];
    for (int k = 0; k < nv; k++) s.M[i][k] = d.M[i * nv + k];
  }
  for (int i = 0; i < m.nu; i++) s.ctrl[i] = d.ctrl[i];
  s.time = d.time;
  for (int b = 0; b < m.nbody; b++) {
    for (int k = 0; k < 3; k++) {
      s.xpos[b][k] = d.xpos[3 * b + k]; s.xipos[b][k] = d.xipos[3 * b + k]; s.subtree_com[b][k] = d.subtree_com[3 * b + k];
    }
    for (int k = 0; k < 4; k++) s.xquat[b][k] = d.xquat[4 * b + k];
    for (int k = 0; k < 6; k++) s.cvel[b][k] = d.cvel[6 * b + k];
    for (int k = 0; k < 10; k++) s.cinert[b][k] = d.cinert[10 * b + k];
  }
  for (int i = 0; i < m.nsensordata; i++) s.sensordata[i] = d.sensordata[i];
  s.ncon = (int)d.contact.size();
  for (int c = 0; c < s.ncon && c < ORC_MAXCON; c++) {
    s.con_dist[c] = d.contact[c].dist;
    for (int k = 0; k < 3; k++) s.con_pos[c][k] = d.contact[c].pos[k];
    for (int k = 0; k < 9; k++) s.con_frame[c][k] = d.contact[c].frame[k];
    s.con_geom[c][0] = d.contact[c].geom1; s.con_geom[c][1] = d.contact[c].geom2;
  }
  s.nefc = d.nefc;
  for (int r = 0; r < d.nefc && r < ORC_MAXEFC; r++) {
    s.efc_force[r] = d.efc_force[r]; s.efc_D[r] = d.efc_D[r]; s.efc_aref[r] = d.efc_aref[r];
    s.efc_pos[r] = d.efc_pos[r]; s.efc_type[r] = d.efc_type[r];
  }
  s.niter = d.solver_niter;
}

template <class R> int run(const mjlModelDesc* m, orcState* s, int mode, int nstep) {
  oracle::Data<R> d;
  load(*m, *s, d);
  for (int i = 0; i < nstep; i++) {
    if (mode == 0) oracle::forward(*m, d); else oracle::step(*m, d);
  }
  save(*m, d, *s);
  return 0;
}

template <class R> int env_reset(const mjlModelDesc* m, const mjlEnvConfig* c, orcState* s, double* aux,
                                 const double* u, double* obs) {
  oracle::Data<R> d;
  R ur[MJL_MAXQ + MJL_MAXV + 2], a[MJL_AUX_DIM], o[MJL_MAXOBS];
  for (int i = 0; i < m->nq - 7 + m->nv + 2; i++) ur[i] = R(u[i]);
  oracle::env_reset(*m, *c, d, a, ur, o);
  save(*m, d, *s);
  for (int i = 0; i < MJL_AUX_DIM; i++) aux[i] = a[i];
  for (int i = 0; i < c->obs_dim; i++) obs[i] = o[i];
  return 0;
}

template <class R> int env_step(const mjlModelDesc* m, const mjlEnvConfig* c, orcState* s, double* aux,
                                const double* act, double* obs, double* rtt) {
  oracle::Data<R> d;
  load(*m, *s, d);
  R a[MJL_AUX_DIM], ac[MJL_MAXU];
  for (int i = 0; i < MJL_AUX_DIM; i++) a[i] = R(aux[i]);
  for (int i = 0; i < m->nu; i++) ac[i] = R(act[i]);
  oracle::EnvOut<R> out;
  oracle::env_step(*m, *c, d, a, ac, out);
  save(*m, d, *s);
  for (int i = 0; i < MJL_AUX_DIM; i++) aux[i] = a[i];
  for (int i = 0; i < c->obs_dim; i++) obs[i] = out.obs[i];
  rtt[0] = out.reward; rtt[1] = out.terminated; rtt[2] = out.truncated;
  return 0;
}

}  // namespace

extern "C" {

// Diagnostics of the truncated-solve study (physics.hpp kDiag*): flags, and the cost log.
void orc_set_diag(int flags) { oracle::g_diag = flags; }
int orc_take_cost_log(double* buf, int cap) {
  int n = (int)std::min<size_t>(oracle::g_cost_log.size(), (size_t)cap);
  std::copy(oracle::g_cost_log.begin(), oracle::g_cost_log.begin() + n, buf);
  oracle::g_cost_log.clear();
  return n;
}

// mode 0: forward only (mjx.forward); mode 1: step (mjx.step). nstep repeats (state carried).
int orc_run(const mjlModelDesc* m, orcState* s, int mode, int nstep, int use_float) {
  return use_float ? run<float>(m, s, mode, nstep) : run<double>(m, s, mode, nstep);
}

int orc_env_reset(const mjlModelDesc* m, const mjlEnvConfig* c, orcState* s, double* aux, const double* u,
                  double* obs, int use_float) {
  return use_float ? env_reset<float>(m, c, s, aux, u, obs) : env_reset<double>(m, c, s, aux, u, obs);
}

int orc_env_step(const mjlModelDesc* m, const mjlEnvConfig* c, orcState* s, double* aux, const double* act,
                 double* obs, double* rtt, int use_float) {
  return use_float ? env_step<float>(m, c, s, aux, act, obs, rtt) : env_step<double>(m, c, s, aux, act, obs, rtt);
}

// Speed-test semantics (mjx_humanoid_speed_test.py:48-57): fresh data, qvel[0]=vel[i], one step,
// out[i] = qpos[0]. Used as the CPU baseline and as the parity reference of mjl_speedtest_step.
int orc_speedtest(const mjlModelDesc* m, const double* vel, int n, double* out, int use_float) {
  for (int i = 0; i < n; i++) {
    if (use_float) {
      oracle::Data<float> d;
      oracle::make_data(*m, d);
      d.qvel[0] = float(vel[i]);
      oracle::step(*m, d);
      out[i] = d.qpos[0];
    } else {
      oracle::Data<double> d;
      oracle::make_data(*m, d);
      d.qvel[0] = vel[i];
      oracle::step(*m, d);
      out[i] = d.qpos[0];
    }
  }
  return 0;
}

// Trajectory rollout for the CPU baseline: nstep steps with ctrl[t, nu] (row-major), state carried.
int orc_rollout(const mjlModelDesc* m, orcState* s, const double* ctrl, int nstep, int use_float) {
  if (use_float) {
    oracle::Data<float> d;
    load(*m, *s, d);
    for (int t = 0; t < nstep; t++) {
      for (int u = 0; u < m->nu; u++) d.ctrl[u] = float(ctrl[t * m->nu + u]);
      oracle::step(*m, d);
    }
    save(*m, d, *s);
  } else {
    oracle::Data<double> d;
    load(*m, *s, d);
    for (int t = 0; t < nstep; t++) {
      for (int u = 0; u < m->nu; u++) d.ctrl[u] = ctrl[t * m->nu + u];
      oracle::step(*m, d);
    }
    save(*m, d, *s);
  }
  return 0;
}

}  // extern "C"

// ---- exact Jacobians by forward-mode dual numbers (the derivative reference of the HIP adjoint)


namespace {
constexpr int kND = 96;  // seeded inputs: qpos (nq) + qvel (nv) + ctrl/action (nu) + aux (9) <= 96
using Dn = oracle::Dual<kND>;
}  // namespace

extern "C" {

// jac [(nq+nv) x (nq+nv+nu)], row-major: d(qpos', qvel') / d(qpos, qvel, ctrl) of one mjx.step.
// qacc_warmstart is held constant (it only seeds the solver).
int orc_step_jacobian(const mjlModelDesc* m, const orcState* s, double* jac) {
  const int nq = m->nq, nv = m->nv, nu = m->nu, ni = nq + nv + nu;
  if (ni > kND) return -1;
  oracle::Data<Dn> d;
  load(*m, *s, d);
  for (int i = 0; i < nq; i++) d.qpos[i].d[i] = 1.0;
  for (int i = 0; i < nv; i++) d.qvel[i].d[nq + i] = 1.0;
  for (int i = 0; i < nu; i++) d.ctrl[i].d[nq + nv + i] = 1.0;
  oracle::step(*m, d);
  for (int i = 0; i < nq; i++)
    for (int k = 0; k < ni; k++) jac[i * ni + k] = d.qpos[i].d[k];
  for (int i = 0; i < nv; i++)
    for (int k = 0; k < ni; k++) jac[(nq + i) * ni + k] = d.qvel[i].d[k];
  return 0;
}

// Env step (src/envs.py:333-492) Jacobian: rows (qpos', qvel', reward, aux'[9]), columns
// (qpos, qvel, action[nu], aux[9]); jac [(nq+nv+1+9) x (nq+nv+nu+9)], row-major.
int orc_env_step_jacobian(const mjlModelDesc* m, const mjlEnvConfig* c, const orcState* s, const double* aux_in,
                          const double* act, double* jac) {
  const int nq = m->nq, nv = m->nv, nu = m->nu, ni = nq + nv + nu + MJL_AUX_DIM;
  if (ni > kND) return -1;
  oracle::Data<Dn> d;
  load(*m, *s, d);
  Dn aux[MJL_AUX_DIM], a[MJL_MAXU];
  for (int i = 0; i < nq; i++) d.qpos[i].d[i] = 1.0;
  for (int i = 0; i < nv; i++) d.qvel[i].d[nq + i] = 1.0;
  for (int i = 0; i < nu; i++) { a[i] = Dn(act[i]); a[i].d[nq + nv + i] = 1.0; }
  for (int i = 0; i < MJL_AUX_DIM; i++) { aux[i] = Dn(aux_in[i]); aux[i].d[nq + nv + nu + i] = 1.0; }
  oracle::EnvOut<Dn> out;
  oracle::env_step(*m, *c, d, aux, a, out);
  int r = 0;
  for (int i = 0; i < nq; i++, r++)
    for (int k = 0; k < ni; k++) jac[r * ni + k] = d.qpos[i].d[k];
  for (int i = 0; i < nv; i++, r++)
    for (int k = 0; k < ni; k++) jac[r * ni + k] = d.qvel[i].d[k];
  for (int k = 0; k < ni; k++) jac[r * ni + k] = out.reward.d[k];
  r++;
  for (int i = 0; i < MJL_AUX_DIM; i++, r++)
    for (int k = 0; k < ni; k++) jac[r * ni + k] = aux[i].d[k];
  return 0;
}

}  // extern "C"

// The same with the carried warm start as one more state block: jax.grad through the Data carry
// differentiates the next solve's dependence on qacc_warmstart (a truncated solve depends on it).
namespace {
constexpr int kNW = 128;
using Dw = oracle::Dual<kNW>;
}  // namespace

extern "C" {

// rows (qpos', qvel', qacc_warmstart'), columns (qpos, qvel, qacc_warmstart, ctrl)
int orc_step_jacobian_ws(const mjlModelDesc* m, const orcState* s, double* jac) {
  const int nq = m->nq, nv = m->nv, nu = m->nu, ni = nq + 2 * nv + nu;
  if (ni > kNW) return -1;
  oracle::Data<Dw> d;
  load(*m, *s, d);
  for (int i = 0; i < nq; i++) d.qpos[i].d[i] = 1.0;
  for (int i = 0; i < nv; i++) { d.qvel[i].d[nq + i] = 1.0; d.qacc_warmstart[i].d[nq + nv + i] = 1.0; }
  for (int i = 0; i < nu; i++) d.ctrl[i].d[nq + 2 * nv + i] = 1.0;
  oracle::step(*m, d);
  int r = 0;
  for (int i = 0; i < nq; i++, r++)
    for (int k = 0; k < ni; k++) jac[r * ni + k] = d.qpos[i].d[k];
  for (int i = 0; i < nv; i++, r++)
    for (int k = 0; k < ni; k++) jac[r * ni + k] = d.qvel[i].d[k];
  for (int i = 0; i < nv; i++, r++)
    for (int k = 0; k < ni; k++) jac[r * ni + k] = d.qacc_warmstart[i].d[k];
  return 0;
}

// rows (qpos', qvel', qacc_warmstart', reward, aux'), columns (qpos, qvel, qacc_warmstart, action, aux)
int orc_env_step_jacobian_ws(const mjlModelDesc* m, const mjlEnvConfig* c, const orcState* s,
                             const double* aux_in, const double* act, double* jac) {
  const int nq = m->nq, nv = m->nv, nu = m->nu, ni = nq + 2 * nv + nu + MJL_AUX_DIM;
  if (ni > kNW) return -1;
  oracle::Data<Dw> d;
  load(*m, *s, d);
  Dw aux[MJL_AUX_DIM], a[MJL_MAXU];
  for (int i = 0; i < nq; i++) d.qpos[i].d[i] = 1.0;
  for (int i = 0; i < nv; i++) { d.qvel[i].d[nq + i] = 1.0; d.qacc_warmstart[i].d[nq + nv + i] = 1.0; }
  for (int i = 0; i < nu; i++) { a[i] = Dw(act[i]); a[i].d[nq + 2 * nv + i] = 1.0; }
  for (int i = 0; i < MJL_AUX_DIM; i++) { aux[i] = Dw(aux_in[i]); aux[i].d[nq + 2 * nv + nu + i] = 1.0; }
  oracle::EnvOut<Dw> out;
  oracle::env_step(*m, *c, d, aux, a, out);
  int r = 0;
  for (int i = 0; i < nq; i++, r++)
    for (int k = 0; k < ni; k++) jac[r * ni + k] = d.qpos[i].d[k];
  for (int i = 0; i < nv; i++, r++)
    for (int k = 0; k < ni; k++) jac[r * ni + k] = d.qvel[i].d[k];
  for (int i = 0; i < nv; i++, r++)
    for (int k = 0; k < ni; k++) jac[r * ni + k] = d.qacc_warmstart[i].d[k];
  for (int k = 0; k < ni; k++) jac[r * ni + k] = out.reward.d[k];
  r++;
  for (int i = 0; i < MJL_AUX_DIM; i++, r++)
    for (int k = 0; k < ni; k++) jac[r * ni + k] = aux[i].d[k];
  return 0;
}

}  // extern "C"
