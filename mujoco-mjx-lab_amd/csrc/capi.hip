// mjx355 C ABI (include/mjx355.h): model upload, batch state ownership, kernel launches.
// Host side only; the kernels live in step_kernels.hip (same translation unit).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>

#include "step_kernels.hip"
#include "adjoint.hip"
#include "ppo_kernels.hip"
#include "apg_kernels.hip"
#include "ppo_loss_kernels.hip"
#include "twin_kernels.hip"

using namespace mjl;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIPCHK(expr)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) return fail(MJL_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

}  // namespace

struct mjlModel {
  mjlModelDesc desc;
  ModelF mf;
  int nefc_max, ncon_max, nvc;  // nvc: 0 = DHum kernels, 1 = DGen kernels
};

struct mjlBatch {
  const mjlModel* model;
  int device, nenv, store_derived, force_global_rows;
  int simds;  // SIMDs of the device (4 per CU): the largest launch that is one wave per SIMD
  ModelF* d_model;
  mjlEnvConfig* d_env;
  int has_env, obs_dim;
  float* d_state;  // one slab holding every per-env field
  StateBuf s;
  int dim[MJL_NFIELD];
  float* field_ptr[MJL_NFIELD];
  float* d_scratch;
  int scratch_stride, gmax_efc, gmax_con;
  float* d_adj_scratch;  // step VJP: per env row slab + adjoint scratch (allocated on first use)
  int vjp_unrolled;      // MJL_OPT_VJP_UNROLLED
  float* d_unr;          // unrolled VJP: per env solve tape + row accumulators (allocated on first use)
  TapeDims unr_dims;
  int adj_stride, adj_row_floats;
  const unsigned long long* ctr_base;  // device RNG counter base (mjl_batch_set_counter_base), or null
  const uint32_t* reset_keys;           // per-env jax.random reset keys (mjl_env_set_reset_keys), or null
  int key_mode;
  float* d_vtape;  // MJL_OPT_VJP_TAPE: slots x nenv x vtape_stride floats (record / replay), or null
  int vtape_slots, vt_w, vt_a, vt_r, vt_t;
  long long vtape_stride;
  float* d_rs;     // MJL_OPT_RESET_POOL: pool slots (the state fields again, [slots * nenv] rows) + obs
  int* d_pool_ctl;  // [nenv, 2] next slot, filled slots
  int pool_slots;
  StateBuf rs;
  float* rs_obs;
};

extern "C" {

const char* mjl_last_error(void) { return g_err.c_str(); }
#ifndef MJL_SRC_HASH
#define MJL_SRC_HASH "unstamped"
#endif
// "mjx355 <ver> (gfx950) src=<hash>": the hash of the sources this library was built from
// (mjx_amd/_srchash.py, stamped by the Makefile); the loader refuses a stale library
const char* mjl_version(void) { return "mjx355 0.2 (gfx950) src=" MJL_SRC_HASH; }

#ifdef MJL_TIMING
// diagnostic build only: install a device buffer [nenv, 16] of per-phase s_memtime stamps
int mjl_debug_set_stamps(unsigned long long* dev_buf) {
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(mjl::g_stamps), &dev_buf, sizeof(dev_buf)));
  return MJL_OK;
}
#endif

static void q2m_host(const double* q, double* m) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  m[0] = 1 - 2 * (y * y + z * z); m[1] = 2 * (x * y - w * z); m[2] = 2 * (x * z + w * y);
  m[3] = 2 * (x * y + w * z); m[4] = 1 - 2 * (x * x + z * z); m[5] = 2 * (y * z - w * x);
  m[6] = 2 * (x * z - w * y); m[7] = 2 * (y * z + w * x); m[8] = 1 - 2 * (x * x + y * y);
}

int mjl_model_create(const mjlModelDesc* d, mjlModel** out) {
  if (!d || !out) return fail(MJL_ERR_ARG, "null argument");
  *out = nullptr;
  if (d->nbody > MJL_MAXBODY || d->njnt > MJL_MAXJNT || d->nv > MJL_MAXV || d->nq > MJL_MAXQ ||
      d->ngeom > MJL_MAXGEOM || d->nsite > MJL_MAXSITE || d->nu > MJL_MAXU || d->ntendon > MJL_MAXTENDON ||
      d->npair > MJL_MAXPAIR || d->nsensor > MJL_MAXSENSOR || d->nbody < 2 || d->nv < 1)
    return fail(MJL_ERR_UNSUPPORTED, "model sizes exceed kernel capacities");
  if (d->nq - 7 + d->nv + 2 > 64) return fail(MJL_ERR_UNSUPPORTED, "too many reset draws for one wave");
  if (d->solver != MJL_SOLVER_NEWTON && d->solver != MJL_SOLVER_CG)
    return fail(MJL_ERR_UNSUPPORTED, "solver %d not supported (Newton, CG)", d->solver);
  if (d->integrator != MJL_INT_EULER && d->integrator != MJL_INT_IMPLICITFAST)
    return fail(MJL_ERR_UNSUPPORTED, "integrator %d not supported (Euler, implicitfast)", d->integrator);
  mjlModel* M = new (std::nothrow) mjlModel();
  if (!M) return fail(MJL_ERR_ARG, "out of host memory");
  M->desc = *d;
  ModelF& f = M->mf;
  std::memset(&f, 0, sizeof(f));
  f.nq = d->nq; f.nv = d->nv; f.nu = d->nu; f.nbody = d->nbody; f.njnt = d->njnt; f.ngeom = d->ngeom;
  f.nsite = d->nsite; f.ntendon = d->ntendon; f.npair = d->npair; f.nsensor = d->nsensor;
  f.nsensordata = d->nsensordata; f.iterations = d->iterations; f.ls_iterations = d->ls_iterations;
  f.solver = d->solver; f.integrator = d->integrator; f.eulerdamp = d->eulerdamp;
  f.timestep = (float)d->timestep; f.impratio = (float)d->impratio; f.tolerance = (float)d->tolerance;
  f.ls_tolerance = (float)d->ls_tolerance; f.meaninertia = (float)d->meaninertia;
  f.scale = (float)(1.0 / (d->meaninertia * (d->nv > 1 ? d->nv : 1)));
  for (int i = 0; i < 3; i++) f.gravity[i] = (float)d->gravity[i];
  int maxlevel = 0;
  for (int b = 0; b < d->nbody; b++) {
    f.body_parentid[b] = d->body_parentid[b]; f.body_rootid[b] = d->body_rootid[b];
    f.body_jntadr[b] = d->body_jntadr[b]; f.body_jntnum[b] = d->body_jntnum[b];
    f.body_dofadr[b] = d->body_dofadr[b]; f.body_dofnum[b] = d->body_dofnum[b];
    f.body_subtree_end[b] = d->body_subtree_end[b]; f.body_level[b] = d->body_level[b];
    if (d->body_level[b] > maxlevel) maxlevel = d->body_level[b];
    for (int i = 0; i < 3; i++) { f.body_pos[b][i] = (float)d->body_pos[b][i]; f.body_ipos[b][i] = (float)d->body_ipos[b][i]; }
    for (int i = 0; i < 4; i++) f.body_quat[b][i] = (float)d->body_quat[b][i];
    for (int i = 0; i < 6; i++) f.body_inertia[b][i] = (float)d->body_inertia[b][i];
    f.body_mass[b] = (float)d->body_mass[b];
    f.body_invweight0[b][0] = (float)d->body_invweight0[b][0];
    f.body_invweight0[b][1] = (float)d->body_invweight0[b][1];
    if (b > 0 && d->body_parentid[b] >= b) { delete M; return fail(MJL_ERR_ARG, "bodies must be in DFS order"); }
  }
  f.maxlevel = maxlevel;
  for (int b = 1; b < d->nbody; b++)
    if (d->body_parentid[b] == 0) f.root[f.nroot++] = b;
  // dof masks along ancestor chains
  for (int b = 1; b < d->nbody; b++) {
    uint32_t mask = 0;
    for (int bb = b; bb > 0; bb = d->body_parentid[bb])
      for (int k = d->body_dofadr[bb]; k < d->body_dofadr[bb] + d->body_dofnum[bb]; k++) mask |= 1u << k;
    f.body_dofmask[b] = mask;
  }
  for (int b = 1; b < d->nbody; b++) {
    uint32_t anc = 0;
    for (int bb = b; bb > 0; bb = d->body_parentid[bb]) anc |= 1u << bb;
    f.body_ancmask[b] = anc;
    const int p = d->body_parentid[b];
    const bool bfree = d->body_jntnum[b] > 0 && d->jnt_type[d->body_jntadr[b]] == MJL_JNT_FREE;
    if (p > 0) {
      f.body_childmask[p] |= 1u << b;
      if (!bfree) f.body_childmask_nf[p] |= 1u << b;
    }
    float mr = 0.f;  // the same float sum, in the same order, as a loop over the subtree would take
    for (int c = b; c < d->body_subtree_end[b]; c++) mr += f.body_mass[c];
    f.body_rootmass[b] = mr;
  }
  for (int j = 0; j < d->njnt; j++) {
    const int b = d->jnt_bodyid[j];
    f.body_jgather[d->jnt_type[j] == MJL_JNT_FREE ? b : d->body_parentid[b]] |= 1u << j;
  }
  int nlim = 0;
  for (int j = 0; j < d->njnt; j++) {
    if (d->jnt_type[j] != MJL_JNT_FREE && d->jnt_type[j] != MJL_JNT_HINGE) {
      delete M; return fail(MJL_ERR_UNSUPPORTED, "joint type %d not supported", d->jnt_type[j]);
    }
    if (d->jnt_type[j] == MJL_JNT_FREE && d->body_jntadr[d->jnt_bodyid[j]] != j) {
      delete M; return fail(MJL_ERR_UNSUPPORTED, "free joint must be the first joint of its body");
    }
    f.jnt_type[j] = d->jnt_type[j]; f.jnt_qposadr[j] = d->jnt_qposadr[j]; f.jnt_dofadr[j] = d->jnt_dofadr[j];
    f.jnt_limited[j] = d->jnt_limited[j];
    nlim += (d->jnt_limited[j] && d->jnt_type[j] == MJL_JNT_HINGE);
    for (int i = 0; i < 3; i++) { f.jnt_pos[j][i] = (float)d->jnt_pos[j][i]; f.jnt_axis[j][i] = (float)d->jnt_axis[j][i]; }
    f.jnt_range[j][0] = (float)d->jnt_range[j][0]; f.jnt_range[j][1] = (float)d->jnt_range[j][1];
    f.jnt_stiffness[j] = (float)d->jnt_stiffness[j]; f.jnt_margin[j] = (float)d->jnt_margin[j];
    f.jnt_solref[j][0] = (float)d->jnt_solref[j][0]; f.jnt_solref[j][1] = (float)d->jnt_solref[j][1];
    for (int i = 0; i < 5; i++) f.jnt_solimp[j][i] = (float)d->jnt_solimp[j][i];
  }
  int anyd = 0;
  for (int k = 0; k < d->nv; k++) {
    f.dof_bodyid[k] = d->dof_bodyid[k]; f.dof_jntid[k] = d->dof_jntid[k]; f.dof_parentid[k] = d->dof_parentid[k];
    f.dof_damping[k] = (float)d->dof_damping[k]; f.dof_armature[k] = (float)d->dof_armature[k];
    f.dof_invweight0[k] = (float)d->dof_invweight0[k];
    anyd |= d->dof_damping[k] > 0;
  }
  f.any_damping = anyd;
  for (int i = 0; i < d->nq; i++) { f.qpos0[i] = (float)d->qpos0[i]; f.qpos_spring[i] = (float)d->qpos_spring[i]; }
  for (int g = 0; g < d->ngeom; g++) {
    f.geom_type[g] = d->geom_type[g]; f.geom_bodyid[g] = d->geom_bodyid[g];
    double gm[9];
    q2m_host(d->geom_quat[g], gm);
    for (int i = 0; i < 3; i++) {
      f.geom_pos[g][i] = (float)d->geom_pos[g][i];
      f.geom_zaxis[g][i] = (float)gm[3 * i + 2];
      f.geom_size[g][i] = (float)d->geom_size[g][i];
    }
  }
  int ncon_max = 0, nefc_max = nlim;
  for (int p = 0; p < d->npair; p++) {
    int kind = d->pair_kind[p];
    if (kind < MJL_COL_PLANE_SPHERE || kind > MJL_COL_CAPSULE_CAPSULE) {
      delete M; return fail(MJL_ERR_UNSUPPORTED, "collision kind %d not supported", kind);
    }
    if (d->pair_condim[p] != 1 && d->pair_condim[p] != 3) {
      delete M; return fail(MJL_ERR_UNSUPPORTED, "condim %d not supported", d->pair_condim[p]);
    }
    f.pair_geom1[p] = d->pair_geom1[p]; f.pair_geom2[p] = d->pair_geom2[p]; f.pair_kind[p] = kind;
    f.pair_condim[p] = d->pair_condim[p];
    f.pair_mu[p] = (float)d->pair_friction[p][0];
    f.pair_solref[p][0] = (float)d->pair_solref[p][0]; f.pair_solref[p][1] = (float)d->pair_solref[p][1];
    for (int i = 0; i < 5; i++) f.pair_solimp[p][i] = (float)d->pair_solimp[p][i];
    f.pair_includemargin[p] = (float)(d->pair_margin[p] - d->pair_gap[p]);
    int b1 = d->geom_bodyid[d->pair_geom1[p]], b2 = d->geom_bodyid[d->pair_geom2[p]];
    double tran = d->body_invweight0[b1][0] + d->body_invweight0[b2][0];
    if (d->pair_condim[p] == 1) f.pair_invweight[p] = (float)tran;
    else {  // pyramidal: common invweight for every edge (constraint._efc_contact_pyramidal)
      double mu = d->pair_friction[p][0];
      double iw = tran + mu * mu * tran;
      f.pair_invweight[p] = (float)(iw * 2 * mu * mu / d->impratio);
    }
    int nc = kind == MJL_COL_PLANE_CAPSULE ? 2 : 1;
    ncon_max += nc;
    nefc_max += nc * (d->pair_condim[p] == 1 ? 1 : 2 * (d->pair_condim[p] - 1));
  }
  for (int s = 0; s < d->nsite; s++) {
    f.site_bodyid[s] = d->site_bodyid[s];
    double sm[9];
    q2m_host(d->site_quat[s], sm);
    for (int i = 0; i < 9; i++) f.site_mat[s][i] = (float)sm[i];
    for (int i = 0; i < 3; i++) { f.site_pos[s][i] = (float)d->site_pos[s][i]; f.site_size[s][i] = (float)d->site_size[s][i]; }
  }
  for (int u = 0; u < d->nu; u++) {
    int j = d->actuator_trnid[u];
    if (j < 0 || j >= d->njnt || d->jnt_type[j] != MJL_JNT_HINGE) {
      delete M; return fail(MJL_ERR_UNSUPPORTED, "actuator %d: only hinge joint transmission supported", u);
    }
    f.actuator_dof[u] = d->jnt_dofadr[j];
    f.actuator_ctrllimited[u] = d->actuator_ctrllimited[u];
    f.actuator_gear[u] = (float)d->actuator_gear[u];
    f.actuator_ctrlrange[u][0] = (float)d->actuator_ctrlrange[u][0];
    f.actuator_ctrlrange[u][1] = (float)d->actuator_ctrlrange[u][1];
  }
  for (int t = 0; t < d->ntendon; t++) {
    f.tendon_num[t] = d->tendon_num[t]; f.tendon_limited[t] = d->tendon_limited[t];
    for (int w = 0; w < d->tendon_num[t]; w++) {
      int j = d->tendon_jnt[t][w];
      f.tendon_qadr[t][w] = d->jnt_qposadr[j];
      f.tendon_dof[t][w] = d->jnt_dofadr[j];
      f.tendon_coef[t][w] = (float)d->tendon_coef[t][w];
    }
    f.tendon_range[t][0] = (float)d->tendon_range[t][0]; f.tendon_range[t][1] = (float)d->tendon_range[t][1];
    f.tendon_margin[t] = (float)d->tendon_margin[t];
    f.tendon_solref[t][0] = (float)d->tendon_solref[t][0]; f.tendon_solref[t][1] = (float)d->tendon_solref[t][1];
    for (int i = 0; i < 5; i++) f.tendon_solimp[t][i] = (float)d->tendon_solimp[t][i];
    f.tendon_invweight0[t] = (float)d->tendon_invweight0[t];
    nefc_max += d->tendon_limited[t];
  }
  for (int s = 0; s < d->nsensor; s++) {
    if (d->sensor_type[s] != MJL_SENS_TOUCH) { delete M; return fail(MJL_ERR_UNSUPPORTED, "sensor type"); }
    f.sensor_type[s] = d->sensor_type[s]; f.sensor_objid[s] = d->sensor_objid[s]; f.sensor_adr[s] = d->sensor_adr[s];
  }
  // packed per-lane records
  for (int b = 0; b < d->nbody; b++) {
    BodyRec& r = f.brec[b];
    r.parent = d->body_parentid[b]; r.level = d->body_level[b];
    r.jntadr = d->body_jntadr[b]; r.jntnum = d->body_jntnum[b];
    r.dofadr = d->body_dofadr[b]; r.dofnum = d->body_dofnum[b];
    r.subtree_end = d->body_subtree_end[b]; r.rootid = d->body_rootid[b];
    r.isfree = d->body_jntnum[b] > 0 && d->jnt_type[d->body_jntadr[b]] == MJL_JNT_FREE;
    r.qadr = r.isfree ? d->jnt_qposadr[d->body_jntadr[b]] : 0;
    if (r.isfree && d->body_jntnum[b] != 1) {
      delete M; return fail(MJL_ERR_UNSUPPORTED, "a body with a free joint must have no other joint");
    }
    for (int i = 0; i < 3; i++) { r.pos[i] = f.body_pos[b][i]; r.ipos[i] = f.body_ipos[b][i]; }
    for (int i = 0; i < 4; i++) r.quat[i] = f.body_quat[b][i];
    r.mass = f.body_mass[b];
    for (int i = 0; i < 6; i++) r.inertia[i] = f.body_inertia[b][i];
    for (int k = 0; k < 3 && k < d->body_jntnum[b]; k++) {
      const int j = d->body_jntadr[b] + k;
      for (int i = 0; i < 3; i++) { f.bhinge[b][k].pos[i] = f.jnt_pos[j][i]; f.bhinge[b][k].axis[i] = f.jnt_axis[j][i]; }
    }
  }
  for (int g = 0; g < d->ngeom; g++) {
    FrameRec& r = f.frec[g];
    r.body = f.geom_bodyid[g];
    for (int i = 0; i < 3; i++) { r.pos[i] = f.geom_pos[g][i]; r.mat[i] = f.geom_zaxis[g][i]; }
  }
  for (int st = 0; st < d->nsite; st++) {
    FrameRec& r = f.frec[32 + st];
    r.body = f.site_bodyid[st];
    for (int i = 0; i < 3; i++) r.pos[i] = f.site_pos[st][i];
    for (int i = 0; i < 9; i++) r.mat[i] = f.site_mat[st][i];
  }
  for (int j = 0; j < d->njnt; j++) {
    JntRec& r = f.jrec[j];
    for (int i = 0; i < 3; i++) { r.pos[i] = f.jnt_pos[j][i]; r.axis[i] = f.jnt_axis[j][i]; }
    r.qadr = d->jnt_qposadr[j];
    r.qpos0 = f.qpos0[r.qadr];
    r.body = d->jnt_bodyid[j]; r.parent = d->body_parentid[r.body];
    r.isfree = d->jnt_type[j] == MJL_JNT_FREE; r.dofadr = d->jnt_dofadr[j];
  }
  for (int k = 0; k < d->nv; k++) {
    DofRec& r = f.drec[k];
    int j = d->dof_jntid[k];
    r.bodyid = d->dof_bodyid[k]; r.jntid = j; r.rootid = d->body_rootid[r.bodyid];
    r.kfree = d->jnt_type[j] == MJL_JNT_FREE ? k - d->jnt_dofadr[j] : -1;
    uint32_t am = 0;
    for (int a = k; a >= 0; a = d->dof_parentid[a]) am |= 1u << a;
    r.ancmask = am;
    r.qadr_spring = d->jnt_type[j] == MJL_JNT_HINGE ? d->jnt_qposadr[j] : -1;
    r.damping = f.dof_damping[k]; r.armature = f.dof_armature[k];
    r.stiffness = f.jnt_stiffness[j];
    r.qpos_spring = r.qadr_spring >= 0 ? f.qpos_spring[r.qadr_spring] : 0.f;
    r.invweight0 = f.dof_invweight0[k];
  }
  for (int g = 0; g < d->ngeom; g++) f.body_geommask[d->geom_bodyid[g]] |= 1u << g;
  for (int k = 0; k < d->nv; k++)  // descendants-or-self of each dof
    for (int a = k; a >= 0; a = d->dof_parentid[a]) f.dof_descmask[a] |= 1u << k;
  for (int p = 0; p < d->npair; p++) {
    PairRec& r = f.prec[p];
    r.g1 = f.pair_geom1[p]; r.g2 = f.pair_geom2[p]; r.kind = f.pair_kind[p]; r.condim = f.pair_condim[p];
    r.r1 = f.geom_size[r.g1][0]; r.h1 = f.geom_size[r.g1][1];
    r.r2 = f.geom_size[r.g2][0]; r.h2 = f.geom_size[r.g2][1];
    r.includemargin = f.pair_includemargin[p]; r.mu = f.pair_mu[p]; r.invweight = f.pair_invweight[p];
    r.b1 = d->geom_bodyid[r.g1]; r.b2 = d->geom_bodyid[r.g2];
    r.mask1 = f.body_dofmask[r.b1]; r.mask2 = f.body_dofmask[r.b2];
  }
  for (int j = 0; j < d->njnt; j++) {
    LimRec& r = f.jlim[j];
    r.on = f.jnt_limited[j] && f.jnt_type[j] == MJL_JNT_HINGE;
    r.qadr = f.jnt_qposadr[j]; r.dofadr = f.jnt_dofadr[j];
    r.lo = f.jnt_range[j][0]; r.hi = f.jnt_range[j][1]; r.margin = f.jnt_margin[j];
    r.invweight = f.dof_invweight0[r.dofadr];
    for (int i = 0; i < 2; i++) r.solref[i] = f.jnt_solref[j][i];
    for (int i = 0; i < 5; i++) r.solimp[i] = f.jnt_solimp[j][i];
  }
  for (int t = 0; t < d->ntendon; t++) {
    LimRec& r = f.tlim[t];
    r.on = f.tendon_limited[t];
    r.lo = f.tendon_range[t][0]; r.hi = f.tendon_range[t][1]; r.margin = f.tendon_margin[t];
    r.invweight = f.tendon_invweight0[t];
    for (int i = 0; i < 2; i++) r.solref[i] = f.tendon_solref[t][i];
    for (int i = 0; i < 5; i++) r.solimp[i] = f.tendon_solimp[t][i];
  }
  M->nefc_max = nefc_max;
  M->ncon_max = ncon_max;
  // compact kernel instantiation when the model fits the humanoid capacities, generic otherwise
  M->nvc = (d->nv <= DHum::NV && d->nbody <= DHum::NB && d->njnt <= DHum::NJ && d->ngeom <= DHum::NG) ? 0 : 1;
  *out = M;
  return MJL_OK;
}

void mjl_model_destroy(mjlModel* m) { delete m; }
int mjl_model_nefc_max(const mjlModel* m) { return m ? m->nefc_max : -1; }

int mjl_batch_create(const mjlModel* model, int nenv, int device, mjlBatch** out) {
  if (!model || !out || nenv <= 0) return fail(MJL_ERR_ARG, "bad argument");
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(MJL_ERR_NOGPU, "no HIP device available");
  if (device < 0 || device >= ndev) return fail(MJL_ERR_ARG, "device %d out of range", device);
  HIPCHK(hipSetDevice(device));
  mjlBatch* B = new (std::nothrow) mjlBatch();
  if (!B) return fail(MJL_ERR_ARG, "out of host memory");
  std::memset(B, 0, sizeof(*B));
  B->model = model; B->device = device; B->nenv = nenv; B->store_derived = 1;
  {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) ncu = 0;
    B->simds = 4 * ncu;
  }
  const mjlModelDesc& d = model->desc;
  int* dim = B->dim;
  dim[MJL_FIELD_QPOS] = d.nq; dim[MJL_FIELD_QVEL] = d.nv; dim[MJL_FIELD_QACC_WARMSTART] = d.nv;
  dim[MJL_FIELD_TIME] = 1; dim[MJL_FIELD_CTRL] = d.nu; dim[MJL_FIELD_QACC] = d.nv;
  dim[MJL_FIELD_XPOS] = d.nbody * 3; dim[MJL_FIELD_XQUAT] = d.nbody * 4; dim[MJL_FIELD_QFRC_ACTUATOR] = d.nv;
  dim[MJL_FIELD_SENSORDATA] = d.nsensordata > 0 ? d.nsensordata : 1; dim[MJL_FIELD_AUX] = MJL_AUX_DIM;
  dim[MJL_FIELD_STATS] = 4; dim[MJL_FIELD_QFRC_BIAS] = d.nv; dim[MJL_FIELD_QFRC_PASSIVE] = d.nv;
  dim[MJL_FIELD_QFRC_CONSTRAINT] = d.nv; dim[MJL_FIELD_QACC_SMOOTH] = d.nv;
  size_t total = 0;
  for (int f = 0; f < MJL_NFIELD; f++) total += (size_t)dim[f] * nenv;
  hipError_t e = hipMalloc(&B->d_state, total * sizeof(float));
  if (e != hipSuccess) { delete B; return fail(MJL_ERR_HIP, "hipMalloc state: %s", hipGetErrorString(e)); }
  size_t off = 0;
  for (int f = 0; f < MJL_NFIELD; f++) { B->field_ptr[f] = B->d_state + off; off += (size_t)dim[f] * nenv; }
  StateBuf& s = B->s;
  s.qpos = B->field_ptr[MJL_FIELD_QPOS]; s.qvel = B->field_ptr[MJL_FIELD_QVEL];
  s.qacc_warmstart = B->field_ptr[MJL_FIELD_QACC_WARMSTART]; s.time = B->field_ptr[MJL_FIELD_TIME];
  s.ctrl = B->field_ptr[MJL_FIELD_CTRL]; s.aux = B->field_ptr[MJL_FIELD_AUX]; s.qacc = B->field_ptr[MJL_FIELD_QACC];
  s.xpos = B->field_ptr[MJL_FIELD_XPOS]; s.xquat = B->field_ptr[MJL_FIELD_XQUAT];
  s.qfrc_actuator = B->field_ptr[MJL_FIELD_QFRC_ACTUATOR]; s.sensordata = B->field_ptr[MJL_FIELD_SENSORDATA];
  s.stats = B->field_ptr[MJL_FIELD_STATS]; s.qfrc_bias = B->field_ptr[MJL_FIELD_QFRC_BIAS];
  s.qfrc_passive = B->field_ptr[MJL_FIELD_QFRC_PASSIVE]; s.qfrc_constraint = B->field_ptr[MJL_FIELD_QFRC_CONSTRAINT];
  s.qacc_smooth = B->field_ptr[MJL_FIELD_QACC_SMOOTH];
  // make_data: zeros, qpos = qpos0
  e = hipMemset(B->d_state, 0, total * sizeof(float));
  if (e == hipSuccess) {
    float* q = new float[(size_t)d.nq * nenv];
    for (int i = 0; i < nenv; i++)
      for (int k = 0; k < d.nq; k++) q[(size_t)i * d.nq + k] = (float)d.qpos0[k];
    e = hipMemcpy(s.qpos, q, sizeof(float) * d.nq * nenv, hipMemcpyHostToDevice);
    delete[] q;
  }
  if (e == hipSuccess) e = hipMalloc(&B->d_model, sizeof(ModelF));
  if (e == hipSuccess) e = hipMemcpy(B->d_model, &model->mf, sizeof(ModelF), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMalloc(&B->d_env, sizeof(mjlEnvConfig));
  // global overflow rows for envs whose active constraints exceed the LDS capacity
  int LD = model->nvc == 0 ? DHum::LD : DGen::LD;
  B->gmax_efc = model->nefc_max > 0 ? model->nefc_max : 1;
  B->gmax_con = model->ncon_max > 0 ? model->ncon_max : 1;
  B->scratch_stride = B->gmax_efc * (LD + 8) + B->gmax_con * (CONW + 2);
  B->scratch_stride = (B->scratch_stride + 3) & ~3;
  if (e == hipSuccess) e = hipMalloc(&B->d_scratch, (size_t)B->scratch_stride * nenv * sizeof(float));
  if (e != hipSuccess) {
    (void)hipFree(B->d_state); (void)hipFree(B->d_model); (void)hipFree(B->d_env); (void)hipFree(B->d_scratch);
    delete B;
    return fail(MJL_ERR_HIP, "batch allocation: %s", hipGetErrorString(e));
  }
  *out = B;
  return MJL_OK;
}

void mjl_batch_destroy(mjlBatch* B) {
  if (!B) return;
  (void)hipSetDevice(B->device);
  (void)hipFree(B->d_state); (void)hipFree(B->d_model); (void)hipFree(B->d_env); (void)hipFree(B->d_scratch);
  (void)hipFree(B->d_adj_scratch);
  (void)hipFree(B->d_unr);
  (void)hipFree(B->d_rs); (void)hipFree(B->d_pool_ctl); (void)hipFree(B->d_vtape);
  delete B;
}

int mjl_batch_nenv(const mjlBatch* B) { return B ? B->nenv : -1; }

int mjl_batch_set_option(mjlBatch* B, int option, int value) {
  if (!B) return fail(MJL_ERR_ARG, "null batch");
  if (option == MJL_OPT_STORE_DERIVED) { B->store_derived = value != 0; return MJL_OK; }
  if (option == MJL_OPT_FORCE_GLOBAL_ROWS) { B->force_global_rows = value != 0; return MJL_OK; }
  if (option == MJL_OPT_VJP_UNROLLED) {
    if (value && B->model->desc.iterations > 256)
      return fail(MJL_ERR_ARG, "unrolled VJP: %d solver iterations (at most 256 are taped)", B->model->desc.iterations);
    // a zoom line search creates up to 1 + 2 ls_iterations Newton points; the tape holds 64 per search
    if (value && 1 + 2 * B->model->desc.ls_iterations > 64)
      return fail(MJL_ERR_ARG, "unrolled VJP: ls_iterations %d (at most 31: the tape holds 64 line-search points)",
                  B->model->desc.ls_iterations);
    B->vjp_unrolled = value != 0;
    return MJL_OK;
  }
  if (option == MJL_OPT_VJP_TAPE) {
    if (value < 0) return fail(MJL_ERR_ARG, "VJP tape: slots must be >= 0");
    HIPCHK(hipSetDevice(B->device));
    (void)hipFree(B->d_vtape);
    B->d_vtape = nullptr; B->vtape_slots = 0;
    if (!value) return MJL_OK;
    const bool gen = B->model->nvc != 0;
    const int LD = gen ? DGen::LD : DHumV::LD;
    TapeDims td;
    td.init(LD, B->gmax_efc, B->model->desc.iterations);
    const long long r4 = 3;
    B->vt_w = 0;
    B->vt_a = (int)((gen ? slot_w_floats<DGen>() : slot_w_floats<DHumV>()) + r4) & ~3;
    B->vt_r = (int)((B->vt_a + (gen ? slot_a_floats<DGen>() : slot_a_floats<DHumV>()) + r4) & ~3);
    const long long rows = ((long long)B->gmax_efc * (LD + 8) + (long long)B->gmax_con * (CONW + 2) + r4) & ~r4;
    B->vt_t = (int)(B->vt_r + rows);
    B->vtape_stride = ((long long)B->vt_t + td.tape + r4) & ~r4;
    const size_t bytes = (size_t)value * B->nenv * (size_t)B->vtape_stride * sizeof(float);
    hipError_t e = hipMalloc(&B->d_vtape, bytes);
    if (e != hipSuccess) { B->d_vtape = nullptr; return fail(MJL_ERR_HIP, "VJP tape (%zu bytes): %s", bytes, hipGetErrorString(e)); }
    B->vtape_slots = value;
    return MJL_OK;
  }
  if (option == MJL_OPT_RESET_POOL) {
    if (value < 0 || value > 64) return fail(MJL_ERR_ARG, "reset pool: 0..64 slots per env");
    HIPCHK(hipSetDevice(B->device));
    (void)hipFree(B->d_rs); (void)hipFree(B->d_pool_ctl);
    B->d_rs = nullptr; B->d_pool_ctl = nullptr; B->pool_slots = 0;
    if (!value) return MJL_OK;
    const size_t rows = (size_t)value * B->nenv;
    size_t total = 0;
    for (int f = 0; f < MJL_NFIELD; f++) total += (size_t)B->dim[f] * rows;
    const size_t obs_floats = (size_t)64 * rows;  // obs_dim <= 64 (mjl_env_config)
    hipError_t e = hipMalloc(&B->d_rs, (total + obs_floats) * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&B->d_pool_ctl, (size_t)B->nenv * 2 * sizeof(int));
    if (e == hipSuccess) e = hipMemset(B->d_pool_ctl, 0, (size_t)B->nenv * 2 * sizeof(int));  // empty
    if (e != hipSuccess) {
      (void)hipFree(B->d_rs); (void)hipFree(B->d_pool_ctl);
      B->d_rs = nullptr; B->d_pool_ctl = nullptr;
      return fail(MJL_ERR_HIP, "reset pool: %s", hipGetErrorString(e));
    }
    float* f[MJL_NFIELD];
    size_t off = 0;
    for (int k = 0; k < MJL_NFIELD; k++) { f[k] = B->d_rs + off; off += (size_t)B->dim[k] * rows; }
    StateBuf& r = B->rs;
    r.qpos = f[MJL_FIELD_QPOS]; r.qvel = f[MJL_FIELD_QVEL]; r.qacc_warmstart = f[MJL_FIELD_QACC_WARMSTART];
    r.time = f[MJL_FIELD_TIME]; r.ctrl = f[MJL_FIELD_CTRL]; r.aux = f[MJL_FIELD_AUX]; r.qacc = f[MJL_FIELD_QACC];
    r.xpos = f[MJL_FIELD_XPOS]; r.xquat = f[MJL_FIELD_XQUAT]; r.qfrc_actuator = f[MJL_FIELD_QFRC_ACTUATOR];
    r.sensordata = f[MJL_FIELD_SENSORDATA]; r.stats = f[MJL_FIELD_STATS]; r.qfrc_bias = f[MJL_FIELD_QFRC_BIAS];
    r.qfrc_passive = f[MJL_FIELD_QFRC_PASSIVE]; r.qfrc_constraint = f[MJL_FIELD_QFRC_CONSTRAINT];
    r.qacc_smooth = f[MJL_FIELD_QACC_SMOOTH];
    B->rs_obs = B->d_rs + total;
    B->pool_slots = value;
    return MJL_OK;
  }
  return fail(MJL_ERR_ARG, "unknown option %d", option);
}

}  // extern "C"

__global__ void masked_copy_kernel(float* dst, const float* src, const float* mask, int nenv, int dim) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long n = (long)nenv * dim;
  if (i >= n) return;
  int env = (int)(i / dim);
  if (!mask || mask[env] > 0.5f) dst[i] = src[i];
}

extern "C" int mjl_get(mjlBatch* B, int field, float* dst, void* stream) {
  if (!B || !dst || field < 0 || field >= MJL_NFIELD) return fail(MJL_ERR_ARG, "bad argument");
  HIPCHK(hipSetDevice(B->device));
  HIPCHK(hipMemcpyAsync(dst, B->field_ptr[field], sizeof(float) * (size_t)B->dim[field] * B->nenv,
                        hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return MJL_OK;
}

extern "C" int mjl_set(mjlBatch* B, int field, const float* src, const float* mask, void* stream) {
  if (!B || !src || field < 0 || field >= MJL_NFIELD) return fail(MJL_ERR_ARG, "bad argument");
  HIPCHK(hipSetDevice(B->device));
  long n = (long)B->dim[field] * B->nenv;
  if (!mask) {
    HIPCHK(hipMemcpyAsync(B->field_ptr[field], src, sizeof(float) * n, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  } else {
    int threads = 256;
    long blocks = (n + threads - 1) / threads;
    hipLaunchKernelGGL(masked_copy_kernel, dim3((unsigned)blocks), dim3(threads), 0, (hipStream_t)stream,
                       B->field_ptr[field], src, mask, B->nenv, B->dim[field]);
    HIPCHK(hipGetLastError());
  }
  return MJL_OK;
}

// packed persistent state rows [qpos | qvel | qacc_warmstart | aux | time] (APG tape)
__global__ void pack_state_kernel(StateBuf S, int nenv, int nq, int nv, float* __restrict__ dst) {
  const int w = nq + 2 * nv + MJL_AUX_DIM + 1;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)nenv * w) return;
  const int e = (int)(t / w), k = (int)(t % w);
  float v;
  if (k < nq) v = S.qpos[(size_t)e * nq + k];
  else if (k < nq + nv) v = S.qvel[(size_t)e * nv + k - nq];
  else if (k < nq + 2 * nv) v = S.qacc_warmstart[(size_t)e * nv + k - nq - nv];
  else if (k < nq + 2 * nv + MJL_AUX_DIM) v = S.aux[(size_t)e * MJL_AUX_DIM + k - nq - 2 * nv];
  else v = S.time[e];
  dst[t] = v;
}
__global__ void unpack_state_kernel(StateBuf S, int nenv, int nq, int nv, const float* __restrict__ src,
                                    const float* __restrict__ ws_src) {
  const int w = nq + 2 * nv + MJL_AUX_DIM + 1;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)nenv * w) return;
  const int e = (int)(t / w), k = (int)(t % w);
  const float v = src[t];
  if (k < nq) S.qpos[(size_t)e * nq + k] = v;
  else if (k < nq + nv) S.qvel[(size_t)e * nv + k - nq] = v;
  else if (k < nq + 2 * nv) S.qacc_warmstart[(size_t)e * nv + k - nq - nv] = ws_src ? ws_src[t] : v;
  else if (k < nq + 2 * nv + MJL_AUX_DIM) S.aux[(size_t)e * MJL_AUX_DIM + k - nq - 2 * nv] = v;
  else S.time[e] = v;
}

extern "C" int mjl_state_size(const mjlBatch* B) {
  if (!B) return -1;
  return B->model->desc.nq + 2 * B->model->desc.nv + MJL_AUX_DIM + 1;
}

extern "C" int mjl_get_state(mjlBatch* B, float* dst, void* stream) {
  if (!B || !dst) return fail(MJL_ERR_ARG, "bad argument");
  HIPCHK(hipSetDevice(B->device));
  const int nq = B->model->desc.nq, nv = B->model->desc.nv;
  const long n = (long)B->nenv * (nq + 2 * nv + MJL_AUX_DIM + 1);
  hipLaunchKernelGGL(pack_state_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, B->s,
                     B->nenv, nq, nv, dst);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

extern "C" int mjl_set_state(mjlBatch* B, const float* src, const float* ws_src, void* stream) {
  if (!B || !src) return fail(MJL_ERR_ARG, "bad argument");
  HIPCHK(hipSetDevice(B->device));
  const int nq = B->model->desc.nq, nv = B->model->desc.nv;
  const long n = (long)B->nenv * (nq + 2 * nv + MJL_AUX_DIM + 1);
  hipLaunchKernelGGL(unpack_state_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, B->s,
                     B->nenv, nq, nv, src, ws_src);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

static KParams make_params(mjlBatch* B) {
  KParams P;
  std::memset(&P, 0, sizeof(P));
  P.pool_slot = -1;
  P.m = B->d_model;
  P.env = B->d_env;
  P.s = B->s;
  P.nenv = B->nenv;
  P.store_derived = B->store_derived;
  P.force_global_rows = B->force_global_rows;
  P.scratch = B->d_scratch;
  P.scratch_stride = B->scratch_stride;
  P.gmax_efc = B->gmax_efc;
  P.gmax_con = B->gmax_con;
  P.ctr_base = B->ctr_base;
  P.keys = B->reset_keys;
  P.key_mode = B->key_mode;
  return P;
}

// env-step launches of at most one wave per SIMD (nenv <= 4 x CUs: C3's 1024-env rollout) take the
// one-wave instantiation (MJL_ONE_WAVE=0 disables it, for A/B runs). Measured (profiles/r4_onewave_ab.jsonl,
// interleaved): pooled env step at 1024 envs 81.4 -> 77.0 us, in-place 109.5 -> 106.4 us; the speed test
// at 1024 envs ran 2 % slower one-wave (55.6 -> 56.7 us), so it keeps the two-wave kernel.
static bool one_wave_launch(const mjlBatch* B) {
  static const bool on = [] { const char* e = std::getenv("MJL_ONE_WAVE"); return !(e && e[0] == '0'); }();
  return on && B->nenv <= B->simds;
}

template <int MODE> static int launch(mjlBatch* B, const KParams& P, void* stream) {
  HIPCHK(hipSetDevice(B->device));
  dim3 grid(B->nenv), block(64);
  constexpr bool kOneWave = MODE == MODE_ENV_STEP;
  if (B->model->nvc == 0 && kOneWave && one_wave_launch(B))
    hipLaunchKernelGGL((step_kernel<DHum, MODE, kOneWave ? 1 : MJL_MINWAVES>), grid, block, 0, (hipStream_t)stream, P);
  else if (B->model->nvc == 0)
    hipLaunchKernelGGL((step_kernel<DHum, MODE>), grid, block, 0, (hipStream_t)stream, P);
  else
    hipLaunchKernelGGL((step_kernel<DGen, MODE>), grid, block, 0, (hipStream_t)stream, P);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

extern "C" {

int mjl_forward(mjlBatch* B, const float* mask, void* stream) {
  if (!B) return fail(MJL_ERR_ARG, "null batch");
  KParams P = make_params(B);
  P.mask = mask;
  return launch<MODE_FORWARD>(B, P, stream);
}

int mjl_step(mjlBatch* B, const float* ctrl, void* stream) {
  if (!B) return fail(MJL_ERR_ARG, "null batch");
  KParams P = make_params(B);
  P.in_ctrl = ctrl;
  return launch<MODE_STEP>(B, P, stream);
}

int mjl_speedtest_step(mjlBatch* B, const float* vel, float* out, void* stream) {
  if (!B || !vel || !out) return fail(MJL_ERR_ARG, "bad argument");
  KParams P = make_params(B);
  P.vel = vel;
  P.out_speed = out;
  P.store_derived = 0;
  return launch<MODE_SPEEDTEST>(B, P, stream);
}

int mjl_env_config(mjlBatch* B, const mjlEnvConfig* cfg) {
  if (!B || !cfg) return fail(MJL_ERR_ARG, "bad argument");
  const mjlModelDesc& d = B->model->desc;
  if (cfg->obs_dim <= 0 || cfg->obs_dim > 64) return fail(MJL_ERR_ARG, "obs_dim must be in 1..64");
  if (cfg->obs_dim != 1 + 3 + (d.nq - 7) + d.nv + 2) return fail(MJL_ERR_ARG, "obs_dim does not match the model");
  if (cfg->pelvis_body_id <= 0 || cfg->pelvis_body_id >= d.nbody || cfg->head_body_id <= 0 ||
      cfg->head_body_id >= d.nbody)
    return fail(MJL_ERR_ARG, "pelvis/head body id out of range");
  if (cfg->touch_sensor_right_id < 0 || cfg->touch_sensor_right_id >= d.nsensordata ||
      cfg->touch_sensor_left_id < 0 || cfg->touch_sensor_left_id >= d.nsensordata)
    return fail(MJL_ERR_ARG, "touch sensor id out of range");
  if (d.nbody < 2 || d.jnt_type[0] != MJL_JNT_FREE) return fail(MJL_ERR_UNSUPPORTED, "env needs a free-floating root");
  // the flip tables must be permutations: the action VJP writes each source's cotangent once
  // (adjoint.hip, o_ctrl[act_perm[lane]]), which covers every entry only for a bijection
  unsigned long long seen = 0;
  for (int i = 0; i < d.nu; i++) {
    if (cfg->act_perm[i] < 0 || cfg->act_perm[i] >= d.nu) return fail(MJL_ERR_ARG, "act_perm out of range");
    seen |= 1ull << cfg->act_perm[i];
  }
  if (seen != (d.nu == 64 ? ~0ull : (1ull << d.nu) - 1)) return fail(MJL_ERR_ARG, "act_perm is not a permutation");
  seen = 0;
  for (int i = 0; i < cfg->obs_dim; i++) {
    if (cfg->obs_perm[i] < 0 || cfg->obs_perm[i] >= cfg->obs_dim) return fail(MJL_ERR_ARG, "obs_perm out of range");
    seen |= 1ull << cfg->obs_perm[i];
  }
  if (seen != (cfg->obs_dim == 64 ? ~0ull : (1ull << cfg->obs_dim) - 1))
    return fail(MJL_ERR_ARG, "obs_perm is not a permutation");
  HIPCHK(hipSetDevice(B->device));
  HIPCHK(hipMemcpy(B->d_env, cfg, sizeof(mjlEnvConfig), hipMemcpyHostToDevice));
  if (B->d_pool_ctl) HIPCHK(hipMemset(B->d_pool_ctl, 0, (size_t)B->nenv * 2 * sizeof(int)));  // drawn under the old config
  B->has_env = 1;
  B->obs_dim = cfg->obs_dim;
  return MJL_OK;
}

int mjl_env_step(mjlBatch* B, const float* act, float* obs, float* rew, float* term, float* trunc, int auto_reset,
                 uint64_t seed, uint64_t counter, void* stream) {
  if (!B || !act || !obs || !rew || !term || !trunc) return fail(MJL_ERR_ARG, "bad argument");
  if (!B->has_env) return fail(MJL_ERR_ARG, "mjl_env_config not called");
  KParams P = make_params(B);
  P.in_ctrl = act; P.obs = obs; P.rew = rew; P.term = term; P.trunc = trunc;
  P.auto_reset = auto_reset;
  P.seed_lo = (uint32_t)seed; P.seed_hi = (uint32_t)(seed >> 32);
  P.ctr_lo = (uint32_t)counter; P.ctr_hi = (uint32_t)(counter >> 32);
  if (B->d_pool_ctl && auto_reset) { P.rs = B->rs; P.rs_obs = B->rs_obs; P.pool_ctl = B->d_pool_ctl; }
  return launch<MODE_ENV_STEP>(B, P, stream);
}

int mjl_env_fill_reset_pool(mjlBatch* B, const int* dev_n, uint64_t seed, uint64_t counter, void* stream) {
  if (!B || !dev_n) return fail(MJL_ERR_ARG, "bad argument");
  if (!B->has_env) return fail(MJL_ERR_ARG, "mjl_env_config not called");
  if (!B->d_pool_ctl) return fail(MJL_ERR_ARG, "MJL_OPT_RESET_POOL not set");
  if (B->reset_keys) return fail(MJL_ERR_ARG, "resets drawn from jax.random keys are not pooled");
  for (int j = 0; j < B->pool_slots; j++) {  // one launch per slot: each uses the batch's per-env scratch
    KParams P = make_params(B);
    const size_t rows = (size_t)j * B->nenv;
    StateBuf& r = P.s;
    r = B->rs;
    r.qpos += rows * B->dim[MJL_FIELD_QPOS]; r.qvel += rows * B->dim[MJL_FIELD_QVEL];
    r.qacc_warmstart += rows * B->dim[MJL_FIELD_QACC_WARMSTART]; r.time += rows * B->dim[MJL_FIELD_TIME];
    r.ctrl += rows * B->dim[MJL_FIELD_CTRL]; r.aux += rows * B->dim[MJL_FIELD_AUX];
    r.qacc += rows * B->dim[MJL_FIELD_QACC]; r.xpos += rows * B->dim[MJL_FIELD_XPOS];
    r.xquat += rows * B->dim[MJL_FIELD_XQUAT]; r.qfrc_actuator += rows * B->dim[MJL_FIELD_QFRC_ACTUATOR];
    r.sensordata += rows * B->dim[MJL_FIELD_SENSORDATA]; r.stats += rows * B->dim[MJL_FIELD_STATS];
    r.qfrc_bias += rows * B->dim[MJL_FIELD_QFRC_BIAS]; r.qfrc_passive += rows * B->dim[MJL_FIELD_QFRC_PASSIVE];
    r.qfrc_constraint += rows * B->dim[MJL_FIELD_QFRC_CONSTRAINT];
    r.qacc_smooth += rows * B->dim[MJL_FIELD_QACC_SMOOTH];
    P.obs = B->rs_obs + rows * B->obs_dim;
    P.pool_ctl = B->d_pool_ctl; P.pool_n = dev_n; P.pool_slot = j; P.pool_slots = B->pool_slots;
    P.store_derived = 1;  // the consuming step may store derived fields
    // a counter domain of its own, the slot in bits 48..55: slot j + T of one rollout and slot j of the
    // next (counter + T) stay distinct for any rollout length T
    const uint64_t c = (counter + ((uint64_t)j << 48)) ^ (1ull << 63);
    P.seed_lo = (uint32_t)seed; P.seed_hi = (uint32_t)(seed >> 32);
    P.ctr_lo = (uint32_t)c; P.ctr_hi = (uint32_t)(c >> 32);
    int rc = launch<MODE_ENV_RESET>(B, P, stream);
    if (rc != MJL_OK) return rc;
  }
  return MJL_OK;
}

int mjl_batch_set_counter_base(mjlBatch* B, const uint64_t* dev_counter_base) {
  if (!B) return fail(MJL_ERR_ARG, "null batch");
  B->ctr_base = (const unsigned long long*)dev_counter_base;
  return MJL_OK;
}

int mjl_env_set_reset_keys(mjlBatch* B, const uint32_t* dev_keys, int mode) {
  if (!B) return fail(MJL_ERR_ARG, "null batch");
  if (dev_keys && mode != MJL_RNG_JAX_PARTITIONABLE && mode != MJL_RNG_JAX_ORIGINAL)
    return fail(MJL_ERR_ARG, "unknown key mode %d", mode);
  B->reset_keys = dev_keys;
  B->key_mode = mode;
  return MJL_OK;
}

int mjl_env_reset(mjlBatch* B, const float* mask, uint64_t seed, uint64_t counter, const float* noise, float* obs,
                  void* stream) {
  if (!B) return fail(MJL_ERR_ARG, "null batch");
  if (!B->has_env) return fail(MJL_ERR_ARG, "mjl_env_config not called");
  KParams P = make_params(B);
  P.mask = mask; P.noise = noise; P.obs = obs;
  P.seed_lo = (uint32_t)seed; P.seed_hi = (uint32_t)(seed >> 32);
  P.ctr_lo = (uint32_t)counter; P.ctr_hi = (uint32_t)(counter >> 32);
  return launch<MODE_ENV_RESET>(B, P, stream);
}

}  // extern "C"

// ---------------------------------------------------------------- step VJP (APG backward)
template <bool ENV, int TM = 0> static int launch_vjp(mjlBatch* B, const VjpArgs& V0, void* stream,
                                                     const KParams* P0 = nullptr) {
  HIPCHK(hipSetDevice(B->device));
  if (!B->d_adj_scratch) {
    const int LD = B->model->nvc == 0 ? DHum::LD : DGen::LD;
    B->adj_row_floats = B->gmax_efc * (LD + 8) + B->gmax_con * (CONW + 2);
    B->adj_row_floats = (B->adj_row_floats + 3) & ~3;
    B->adj_stride = B->adj_row_floats + adj_scratch_floats(B->gmax_efc, B->gmax_con);
    if (B->model->nvc == 0) B->adj_stride += DHumV::NV * DHumV::LD;  // lean unrolled replay: M-bar rows
    B->adj_stride = (B->adj_stride + 3) & ~3;
    hipError_t e = hipMalloc(&B->d_adj_scratch, (size_t)B->adj_stride * B->nenv * sizeof(float));
    if (e != hipSuccess) { B->d_adj_scratch = nullptr; return fail(MJL_ERR_HIP, "adjoint scratch: %s", hipGetErrorString(e)); }
  }
  if (B->vjp_unrolled && !B->d_unr) {
    B->unr_dims.init(B->model->nvc == 0 ? DHum::LD : DGen::LD, B->gmax_efc, B->model->desc.iterations);
    hipError_t e = hipMalloc(&B->d_unr, (size_t)B->unr_dims.stride * B->nenv * sizeof(float));
    if (e != hipSuccess) { B->d_unr = nullptr; return fail(MJL_ERR_HIP, "unrolled VJP tape: %s", hipGetErrorString(e)); }
  }
  KParams P = P0 ? *P0 : make_params(B);
  VjpArgs V = V0;
  V.unr = B->vjp_unrolled ? B->d_unr : nullptr;
  V.slot_stride = B->vtape_stride;
  V.s_w = B->vt_w; V.s_a = B->vt_a; V.s_r = B->vt_r; V.s_t = B->vt_t;
  V.td = B->unr_dims;
  V.scratch = B->d_adj_scratch;
  V.scratch_stride = B->adj_stride;
  V.row_floats = B->adj_row_floats;
  dim3 grid(B->nenv), block(64);
  // the replay on the humanoid dims takes the lean layout (20 KB of LDS: one round of 8 envs per CU;
  // MJL_VJP_LEAN=0 keeps the full one, for A/B)
  static const bool lean_ok = [] { const char* e = std::getenv("MJL_VJP_LEAN"); return !(e && e[0] == '0'); }();
  if constexpr (TM == 2) {
    // (unrolled: CG only -- its reverse sweep refactors nothing; Newton's per-iteration Hessian factors
    // need the full layout's LDS)
    if (B->model->nvc == 0 && (!B->vjp_unrolled || B->model->desc.solver == MJL_SOLVER_CG) && lean_ok) {
      hipLaunchKernelGGL((vjp_kernel<DHumV, ENV, TM, true>), grid, block, 0, (hipStream_t)stream, P, V);
      HIPCHK(hipGetLastError());
      return MJL_OK;
    }
  }
  // the implicit record on the humanoid dims keeps its rows in LDS (vjp_record_kernel, the same slot as
  // vjp_kernel's record); MJL_OPT_FORCE_GLOBAL_ROWS keeps the global-row record (A/B, parity tests)
  if constexpr (TM == 1 && ENV) {
    if (B->model->nvc == 0 && !B->force_global_rows) {
      if (B->vjp_unrolled)
        hipLaunchKernelGGL((vjp_record_kernel<DHum, DHumV, true>), grid, block, 0, (hipStream_t)stream, P, V);
      else
        hipLaunchKernelGGL((vjp_record_kernel<DHum, DHumV>), grid, block, 0, (hipStream_t)stream, P, V);
      HIPCHK(hipGetLastError());
      return MJL_OK;
    }
    if (V.post.alive) {  // the other record kernels leave the post-step update to its own launch
      VjpArgs V2 = V;
      V2.post.alive = nullptr;
      if (B->model->nvc == 0)
        hipLaunchKernelGGL((vjp_kernel<DHumV, ENV, TM>), grid, block, 0, (hipStream_t)stream, P, V2);
      else
        hipLaunchKernelGGL((vjp_kernel<DGen, ENV, TM>), grid, block, 0, (hipStream_t)stream, P, V2);
      HIPCHK(hipGetLastError());
      hipLaunchKernelGGL(apg_post_kernel, dim3((B->nenv + kPostEnvs - 1) / kPostEnvs), dim3(64 * kPostEnvs), 0,
                         (hipStream_t)stream, B->s, B->model->desc.nq, B->model->desc.nv, P.rew, P.term, P.trunc,
                         V.post);
      HIPCHK(hipGetLastError());
      return MJL_OK;
    }
  }
  if (B->model->nvc == 0)
    hipLaunchKernelGGL((vjp_kernel<DHumV, ENV, TM>), grid, block, 0, (hipStream_t)stream, P, V);
  else
    hipLaunchKernelGGL((vjp_kernel<DGen, ENV, TM>), grid, block, 0, (hipStream_t)stream, P, V);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

extern "C" {

int mjl_step_vjp(mjlBatch* B, const float* g_qpos, const float* g_qvel, float* out_qpos, float* out_qvel,
                 float* out_ctrl, void* stream) {
  if (!B || !g_qpos || !g_qvel || !out_qpos || !out_qvel || !out_ctrl) return fail(MJL_ERR_ARG, "bad argument");
  VjpArgs V;
  std::memset(&V, 0, sizeof(V));
  V.g_qpos = g_qpos; V.g_qvel = g_qvel; V.o_qpos = out_qpos; V.o_qvel = out_qvel; V.o_ctrl = out_ctrl;
  return launch_vjp<false>(B, V, stream);
}

int mjl_env_step_vjp(mjlBatch* B, const float* act, const float* g_qpos, const float* g_qvel, const float* g_rew,
                     const float* g_aux, float* out_qpos, float* out_qvel, float* out_act, float* out_aux,
                     void* stream) {
  return mjl_env_step_vjp_guarded(B, act, g_qpos, g_qvel, g_rew, g_aux, out_qpos, out_qvel, out_act, out_aux, nullptr,
                                  stream);
}

int mjl_env_step_vjp_guarded(mjlBatch* B, const float* act, const float* g_qpos, const float* g_qvel,
                             const float* g_rew, const float* g_aux, float* out_qpos, float* out_qvel,
                             float* out_act, float* out_aux, float* nonfinite_count, void* stream) {
  if (!B || !act || !g_qpos || !g_qvel || !g_rew || !g_aux || !out_qpos || !out_qvel || !out_act || !out_aux)
    return fail(MJL_ERR_ARG, "bad argument");
  if (!B->has_env) return fail(MJL_ERR_ARG, "mjl_env_config not called");
  VjpArgs V;
  std::memset(&V, 0, sizeof(V));
  V.act = act; V.g_qpos = g_qpos; V.g_qvel = g_qvel; V.g_rew = g_rew; V.g_aux = g_aux;
  V.o_qpos = out_qpos; V.o_qvel = out_qvel; V.o_ctrl = out_act; V.o_aux = out_aux;
  V.nonfinite = nonfinite_count;
  return launch_vjp<true>(B, V, stream);
}

int mjl_step_vjp_full(mjlBatch* B, const float* g_qpos, const float* g_qvel, const float* g_qacc_ws,
                      float* out_qpos, float* out_qvel, float* out_qacc_ws, float* out_ctrl, void* stream) {
  if (!B || !g_qpos || !g_qvel || !out_qpos || !out_qvel || !out_ctrl) return fail(MJL_ERR_ARG, "bad argument");
  VjpArgs V;
  std::memset(&V, 0, sizeof(V));
  V.g_qpos = g_qpos; V.g_qvel = g_qvel; V.o_qpos = out_qpos; V.o_qvel = out_qvel; V.o_ctrl = out_ctrl;
  V.g_ws = g_qacc_ws; V.o_ws = out_qacc_ws;
  return launch_vjp<false>(B, V, stream);
}

int mjl_env_step_vjp_full(mjlBatch* B, const float* act, const float* g_qpos, const float* g_qvel,
                          const float* g_qacc_ws, const float* g_rew, const float* g_aux, float* out_qpos,
                          float* out_qvel, float* out_qacc_ws, float* out_act, float* out_aux,
                          float* nonfinite_count, void* stream) {
  if (!B || !act || !g_qpos || !g_qvel || !g_rew || !g_aux || !out_qpos || !out_qvel || !out_act || !out_aux)
    return fail(MJL_ERR_ARG, "bad argument");
  if (!B->has_env) return fail(MJL_ERR_ARG, "mjl_env_config not called");
  VjpArgs V;
  std::memset(&V, 0, sizeof(V));
  V.act = act; V.g_qpos = g_qpos; V.g_qvel = g_qvel; V.g_rew = g_rew; V.g_aux = g_aux;
  V.o_qpos = out_qpos; V.o_qvel = out_qvel; V.o_ctrl = out_act; V.o_aux = out_aux;
  V.g_ws = g_qacc_ws; V.o_ws = out_qacc_ws;
  V.nonfinite = nonfinite_count;
  return launch_vjp<true>(B, V, stream);
}

int mjl_env_step_record(mjlBatch* B, int slot, const float* act, float* obs, float* rew, float* term, float* trunc,
                        void* stream) {
  if (!B || !act || !obs || !rew || !term || !trunc) return fail(MJL_ERR_ARG, "bad argument");
  if (!B->has_env) return fail(MJL_ERR_ARG, "mjl_env_config not called");
  if (!B->d_vtape || slot < 0 || slot >= B->vtape_slots) return fail(MJL_ERR_ARG, "VJP tape slot %d not allocated", slot);
  KParams P = make_params(B);
  P.obs = obs; P.rew = rew; P.term = term; P.trunc = trunc;
  VjpArgs V;
  std::memset(&V, 0, sizeof(V));
  V.act = act;
  V.slot = B->d_vtape + (size_t)slot * B->nenv * (size_t)B->vtape_stride;
  return launch_vjp<true, 1>(B, V, stream, &P);
}

int mjl_env_step_record_apg(mjlBatch* B, int slot, const float* act, float* obs, float* rew, float* term, float* trunc,
                            float gamma, float diverge_qvel, uint8_t* alive, float* disc, float* ret, float* dropped,
                            float* grew, float* rfin, void* stream) {
  if (!B || !act || !obs || !rew || !term || !trunc || !alive || !disc || !ret || !dropped || !grew || !rfin)
    return fail(MJL_ERR_ARG, "bad argument");
  if (!B->has_env) return fail(MJL_ERR_ARG, "mjl_env_config not called");
  if (!B->d_vtape || slot < 0 || slot >= B->vtape_slots) return fail(MJL_ERR_ARG, "VJP tape slot %d not allocated", slot);
  KParams P = make_params(B);
  P.obs = obs; P.rew = rew; P.term = term; P.trunc = trunc;
  VjpArgs V;
  std::memset(&V, 0, sizeof(V));
  V.act = act;
  V.slot = B->d_vtape + (size_t)slot * B->nenv * (size_t)B->vtape_stride;
  V.post = ApgPostArgs{gamma, diverge_qvel, alive, disc, ret, dropped, grew, rfin, B->nenv};
  return launch_vjp<true, 1>(B, V, stream, &P);
}

int mjl_env_step_vjp_replay(mjlBatch* B, int slot, const float* act, const float* g_qpos, const float* g_qvel,
                            const float* g_qacc_ws, const float* g_rew, const float* g_aux, float* out_qpos,
                            float* out_qvel, float* out_qacc_ws, float* out_act, float* out_aux,
                            float* nonfinite_count, void* stream) {
  if (!B || !act || !g_qpos || !g_qvel || !g_rew || !g_aux || !out_qpos || !out_qvel || !out_act || !out_aux)
    return fail(MJL_ERR_ARG, "bad argument");
  if (!B->has_env) return fail(MJL_ERR_ARG, "mjl_env_config not called");
  if (!B->d_vtape || slot < 0 || slot >= B->vtape_slots) return fail(MJL_ERR_ARG, "VJP tape slot %d not allocated", slot);
  VjpArgs V;
  std::memset(&V, 0, sizeof(V));
  V.act = act; V.g_qpos = g_qpos; V.g_qvel = g_qvel; V.g_rew = g_rew; V.g_aux = g_aux;
  V.o_qpos = out_qpos; V.o_qvel = out_qvel; V.o_ctrl = out_act; V.o_aux = out_aux;
  V.g_ws = g_qacc_ws; V.o_ws = out_qacc_ws;
  V.nonfinite = nonfinite_count;
  V.slot = B->d_vtape + (size_t)slot * B->nenv * (size_t)B->vtape_stride;
  return launch_vjp<true, 2>(B, V, stream);
}

}  // extern "C"

// ---------------------------------------------------------------- PPO host-loop kernels
extern "C" int mjl_gae(const float* rew, const float* val, const float* term, const float* trunc, int T, int B,
                       double gamma, double lam, float* adv, float* ret, void* stream) {
  if (!rew || !val || !term || !trunc || !adv || !ret || T < 0 || B < 0) return fail(MJL_ERR_ARG, "bad argument");
  if (T == 0 || B == 0) return MJL_OK;
  hipLaunchKernelGGL(gae_kernel, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream, rew, val, term, trunc, T,
                     B, (float)gamma, (float)(gamma * lam), adv, ret);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

extern "C" int mjl_obs_normalize(const float* x, const float* mean, const float* var, int n, int dim, float clip,
                                 float* y, void* stream) {
  if (!x || !mean || !var || !y || n < 0 || dim <= 0) return fail(MJL_ERR_ARG, "bad argument");
  if (n == 0) return MJL_OK;
  const long long tot = (long long)n * dim;
  hipLaunchKernelGGL(obs_normalize_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x,
                     mean, var, n, dim, clip, y);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

extern "C" int mjl_policy_head(const float* z, const float* log_std, const float* eps, int B, int A, float* act,
                               float* logp, void* stream) {
  if (!z || !log_std || !eps || !act || !logp || B < 0 || A <= 0) return fail(MJL_ERR_ARG, "bad argument");
  if (B == 0) return MJL_OK;
  hipLaunchKernelGGL(policy_head_kernel, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream, z, log_std, eps, B,
                     A, act, logp);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

static int policy_dims(int nlayer, const int* dims, PolicyDims& pd) {
  if (nlayer < 1 || nlayer > kPolMaxLayers || !dims) return fail(MJL_ERR_ARG, "policy: 1..%d layers", kPolMaxLayers);
  pd.nlayer = nlayer;
  pd.obs_dim = dims[0];
  pd.act_dim = dims[nlayer];
  long long off = 0;
  for (int l = 0; l < nlayer; l++) {
    if (dims[l] <= 0 || dims[l + 1] <= 0) return fail(MJL_ERR_ARG, "policy: layer sizes must be positive");
    pd.K[l] = (dims[l] + 15) & ~15;
    pd.N[l] = (dims[l + 1] + 15) & ~15;
    if (pd.K[l] > 256 || pd.N[l] > 256) return fail(MJL_ERR_ARG, "policy: layer sizes above 256 not supported");
    pd.off[l] = off;
    off += (long long)pd.K[l] * pd.N[l] + pd.N[l];
  }
  return MJL_OK;
}

extern "C" long long mjl_policy_param_floats(int nlayer, const int* dims) {
  PolicyDims pd;
  if (policy_dims(nlayer, dims, pd) != MJL_OK) return -1;
  const int l = nlayer - 1;
  return pd.off[l] + (long long)pd.K[l] * pd.N[l] + pd.N[l];
}

extern "C" int mjl_policy_fwd(const float* obs, const float* mean, const float* var, float clip, const float* params,
                              int nlayer, const int* dims, const float* log_std, const float* eps, int B, float* act,
                              float* logp, void* stream) {
  if (!obs || !mean || !var || !params || !log_std || !eps || !act || !logp || B < 0)
    return fail(MJL_ERR_ARG, "bad argument");
  PolicyDims pd;
  if (int rc = policy_dims(nlayer, dims, pd)) return rc;
  if (B == 0) return MJL_OK;
  hipLaunchKernelGGL(policy_rollout_kernel, dim3((B + 15) / 16), dim3(64 * kPolWaves), 0, (hipStream_t)stream, obs, mean, var,
                     clip, params, pd, log_std, eps, B, act, logp);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

extern "C" long long mjl_colsum_scratch(int n, int d) {
  if (n <= 0 || d <= 0) return 0;
  const ColsumPlan p(n, d);
  return p.R > 1 ? (long long)p.R * d : 0;
}

// batched plans (nb > 1): the stage-1 chunks must not straddle two matrices, so n % chunk == 0; the
// stage-2 "chunk" is then one matrix's R / nb chunk rows, and stage 2 writes out[b][d] directly
static int batched_plan_ok(int nb, int n, const ColsumPlan& p) { return nb == 1 || (p.R > 1 && n % p.chunk == 0); }

extern "C" long long mjl_colsum_batched_scratch(int nb, int n, int d) {
  if (nb <= 0 || n <= 0 || d <= 0) return 0;
  const ColsumPlan p(n, d);
  return p.R > 1 ? (long long)nb * p.R * d : 0;
}

// first stages only, with the caller's chunk: partials [nb][n / chunk][d] (the twin update reduces
// every layer's partials together afterwards, mjl_slice_sum_multi; 32-row chunks give its 8,192-row
// minibatch 512 blocks per pass where the two-stage plan's 128-row chunks gave 128 for 256 CUs)
extern "C" int mjl_tanh_bwd_colsum_partials(const float* g, const float* y, int nb, int n, int d, int chunk, float* dz,
                                            float* partials, void* stream) {
  if (!g || !y || !dz || !partials || nb <= 0 || n <= 0 || d <= 0 || chunk <= 0 || n % chunk)
    return fail(MJL_ERR_ARG, "bad argument");
  if (d % 4 || ((uintptr_t)g | (uintptr_t)y | (uintptr_t)dz | (uintptr_t)partials) % 16)
    return fail(MJL_ERR_ARG, "tanh_bwd_colsum_partials: d divisible by 4 and 16-byte aligned rows expected");
  const int dq = d / 4 < 64 ? d / 4 : 64;
  hipLaunchKernelGGL(tanh_bwd_colsum_kernel, dim3((unsigned)((d / 4 + dq - 1) / dq), (unsigned)(n / chunk * nb)),
                     dim3(256), 0, (hipStream_t)stream, g, y, n * nb, d, dq, chunk, dz, partials);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

extern "C" int mjl_colsum_batched(const float* x, int nb, int n, int d, float* scratch, float* out, void* stream) {
  if ((!x && n > 0) || !out || nb <= 0 || n < 0 || d <= 0) return fail(MJL_ERR_ARG, "bad argument");
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) {
    HIPCHK(hipMemsetAsync(out, 0, sizeof(float) * (size_t)d * nb, s));
    return MJL_OK;
  }
  const ColsumPlan p(n, d);
  if (!batched_plan_ok(nb, n, p)) return fail(MJL_ERR_ARG, "colsum_batched: n must be a multiple of %d", p.chunk);
  if (p.R > 1 && !scratch) return fail(MJL_ERR_ARG, "colsum needs mjl_colsum_batched_scratch(nb, n, d) floats of scratch");
  const unsigned tiles1 = (unsigned)((d + p.dc1 - 1) / p.dc1);
  hipLaunchKernelGGL(colsum_kernel, dim3(tiles1, (unsigned)(p.R * nb)), dim3(256), 0, s, x, n * nb, d, p.dc1, p.chunk,
                     p.R > 1 ? scratch : out);
  HIPCHK(hipGetLastError());
  if (p.R > 1) {
    const unsigned tiles2 = (unsigned)((d + p.dc2 - 1) / p.dc2);
    hipLaunchKernelGGL(colsum_kernel, dim3(tiles2, (unsigned)nb), dim3(256), 0, s, scratch, p.R * nb, d, p.dc2, p.R,
                       out);
    HIPCHK(hipGetLastError());
  }
  return MJL_OK;
}

extern "C" int mjl_colsum(const float* x, int n, int d, float* scratch, float* out, void* stream) {
  return mjl_colsum_batched(x, 1, n, d, scratch, out, stream);
}

extern "C" int mjl_tanh_bwd_colsum_batched(const float* g, const float* y, int nb, int n, int d, float* dz,
                                           float* scratch, float* colsum_out, void* stream) {
  if (!g || !y || !dz || !colsum_out || nb <= 0 || n <= 0 || d <= 0) return fail(MJL_ERR_ARG, "bad argument");
  if (d % 4 || ((uintptr_t)g | (uintptr_t)y | (uintptr_t)dz | (uintptr_t)colsum_out) % 16)
    return fail(MJL_ERR_ARG, "tanh_bwd_colsum: d divisible by 4 and 16-byte aligned rows expected");
  hipStream_t s = (hipStream_t)stream;
  const ColsumPlan p(n, d);
  if (!batched_plan_ok(nb, n, p)) return fail(MJL_ERR_ARG, "tanh_bwd_colsum_batched: n must be a multiple of %d", p.chunk);
  if (p.R > 1 && (!scratch || (uintptr_t)scratch % 16))
    return fail(MJL_ERR_ARG, "tanh_bwd_colsum needs mjl_colsum_batched_scratch(nb, n, d) floats of 16-byte aligned scratch");
  const int dq = d / 4 < 64 ? d / 4 : 64;
  const unsigned tiles1 = (unsigned)((d / 4 + dq - 1) / dq);
  hipLaunchKernelGGL(tanh_bwd_colsum_kernel, dim3(tiles1, (unsigned)(p.R * nb)), dim3(256), 0, s, g, y, n * nb, d, dq,
                     p.chunk, dz, p.R > 1 ? scratch : colsum_out);
  HIPCHK(hipGetLastError());
  if (p.R > 1) {
    const unsigned tiles2 = (unsigned)((d + p.dc2 - 1) / p.dc2);
    hipLaunchKernelGGL(colsum_kernel, dim3(tiles2, (unsigned)nb), dim3(256), 0, s, scratch, p.R * nb, d, p.dc2, p.R,
                       colsum_out);
    HIPCHK(hipGetLastError());
  }
  return MJL_OK;
}

extern "C" int mjl_tanh_bwd_colsum(const float* g, const float* y, int n, int d, float* dz, float* scratch,
                                   float* colsum_out, void* stream) {
  return mjl_tanh_bwd_colsum_batched(g, y, 1, n, d, dz, scratch, colsum_out, stream);
}

extern "C" int mjl_slice_sum_batched(const float* x, int nb, int ns, long long m, float* out, void* stream) {
  if (!x || !out || nb <= 0 || ns <= 0 || m <= 0) return fail(MJL_ERR_ARG, "bad argument");
  if (m % 4 || ((uintptr_t)x | (uintptr_t)out) % 16)
    return fail(MJL_ERR_ARG, "slice_sum: slice length divisible by 4 and 16-byte aligned buffers expected");
  const long long q = m / 4;
  hipLaunchKernelGGL(slice_sum_kernel, dim3((unsigned)((q + 255) / 256), (unsigned)nb), dim3(256), 0,
                     (hipStream_t)stream, x, ns, m, out);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

extern "C" int mjl_slice_sum_multi(int nseg, const float* const* x, float* const* out, const int* nb, const int* ns,
                                   const long long* m, float* step0, float* step1, int* ctr, void* stream) {
  if (nseg < 1 || nseg > kSliceSegMax || !x || !out || !nb || !ns || !m) return fail(MJL_ERR_ARG, "bad argument");
  SliceSegs sg;
  std::memset(&sg, 0, sizeof(sg));
  sg.nseg = nseg;
  sg.step0 = step0; sg.step1 = step1; sg.ctr = ctr;
  for (int k = 0; k < nseg; k++) {
    if (!x[k] || !out[k] || nb[k] <= 0 || ns[k] <= 0 || m[k] <= 0) return fail(MJL_ERR_ARG, "bad argument");
    sg.x[k] = x[k]; sg.out[k] = out[k]; sg.m[k] = m[k]; sg.ns[k] = ns[k]; sg.nb[k] = nb[k];
    sg.vec[k] = (m[k] % 4 == 0 && ((uintptr_t)x[k] | (uintptr_t)out[k]) % 16 == 0) ? 1 : 0;
    int lanes = 1;  // lanes per output: about 8 slices each, at most a wave
    while (lanes < 64 && ns[k] >= 16 * lanes) lanes *= 2;
    sg.lanes[k] = lanes;
    const long long units = sg.vec[k] ? m[k] / 4 : m[k];
    const long long outs = 256 / lanes;
    const long long blocks = (long long)nb[k] * ((units + outs - 1) / outs);
    if (sg.blk[k] + blocks >= (1LL << 30)) return fail(MJL_ERR_ARG, "slice_sum_multi: too many elements");
    sg.blk[k + 1] = sg.blk[k] + (int)blocks;
  }
  hipLaunchKernelGGL(slice_sum_multi_kernel, dim3((unsigned)sg.blk[nseg]), dim3(256), 0, (hipStream_t)stream, sg);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

extern "C" int mjl_slice_sum(const float* x, int ns, long long m, float* out, void* stream) {
  return mjl_slice_sum_batched(x, 1, ns, m, out, stream);
}

extern "C" int mjl_bias_act(float* x, const float* bias, int nb, long long rows, int n, unsigned act_mask,
                            void* stream) {
  if (!x || !bias || nb <= 0 || rows < 0 || n <= 0) return fail(MJL_ERR_ARG, "bad argument");
  if (rows == 0) return MJL_OK;
  if ((long long)nb * rows * n >= (1LL << 31)) return fail(MJL_ERR_ARG, "bias_act: at most 2^31 elements");
  const bool v4 = n % 4 == 0 && (uintptr_t)x % 16 == 0 && (uintptr_t)bias % 16 == 0;
  const long long groups = (long long)nb * rows * n / (v4 ? 4 : 1);
  const dim3 grid((unsigned)((groups + 255) / 256));
  if (v4)
    hipLaunchKernelGGL(bias_act_kernel<4>, grid, dim3(256), 0, (hipStream_t)stream, x, bias, nb, rows, n, act_mask);
  else
    hipLaunchKernelGGL(bias_act_kernel<1>, grid, dim3(256), 0, (hipStream_t)stream, x, bias, nb, rows, n, act_mask);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

extern "C" int mjl_tanh_inplace(float* x, long long n, void* stream) {
  if (!x || n < 0) return fail(MJL_ERR_ARG, "bad argument");
  if (n % 4 || (uintptr_t)x % 16) return fail(MJL_ERR_ARG, "tanh_inplace: length divisible by 4, 16-byte aligned");
  if (n == 0) return MJL_OK;
  const long long q = n / 4;
  hipLaunchKernelGGL(tanh_inplace_kernel, dim3((unsigned)((q + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, q);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

// jax.random.split over a batch of keys (train_ppo.py:132,150: random.split(rng); random.split(key, num_envs))
__global__ void prng_split_kernel(const uint32_t* __restrict__ keys, int n, int num, int mode, uint32_t* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * num) return;
  const int k = t / num, j = t % num;
  const uint32_t k0 = keys[2 * (size_t)k], k1 = keys[2 * (size_t)k + 1];
  uint32_t o0, o1;
  if (mode == MJL_RNG_JAX_PARTITIONABLE) {
    o0 = 0u; o1 = (uint32_t)j;
    threefry2x32(k0, k1, o0, o1);
  } else {  // words 2j, 2j + 1 of threefry_2x32(key, iota(2 num)): pairs (c, c + num)
    const uint32_t w0 = (uint32_t)(2 * j), w1 = w0 + 1u, h = (uint32_t)num;
    uint32_t a0 = w0 < h ? w0 : w0 - h, a1 = a0 + h, b0 = w1 < h ? w1 : w1 - h, b1 = b0 + h;
    threefry2x32(k0, k1, a0, a1);
    threefry2x32(k0, k1, b0, b1);
    o0 = w0 < h ? a0 : a1;
    o1 = w1 < h ? b0 : b1;
  }
  out[2 * (size_t)t] = o0;
  out[2 * (size_t)t + 1] = o1;
}

extern "C" int mjl_prng_split(const uint32_t* keys, int n, int num, int mode, uint32_t* out, void* stream) {
  if (!keys || !out || n < 0 || num < 1) return fail(MJL_ERR_ARG, "bad argument");
  if (mode != MJL_RNG_JAX_PARTITIONABLE && mode != MJL_RNG_JAX_ORIGINAL) return fail(MJL_ERR_ARG, "unknown key mode %d", mode);
  if (n == 0) return MJL_OK;
  hipLaunchKernelGGL(prng_split_kernel, dim3((n * num + 255) / 256), dim3(256), 0, (hipStream_t)stream, keys, n, num,
                     mode, out);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

// ---------------------------------------------------------------- APG rollout bookkeeping
// U (units per row slot) covers every layer width, and k0 for the backward, whose last layer writes k0
// input cotangents per row (the forward stages its k0 inputs by a loop: 32-unit slots, 8 rows per block,
// for the APG policy's 32-wide layers)
static int small_mlp_setup(int B, int k0, int nl, const int* widths, const float* const* w, const float* const* b,
                           float* const* ys, SmallMlp& P, bool fwd = false) {
  if (B < 0 || nl < 1 || nl > kSmlMaxL || k0 < 1 || k0 > kSmlMaxW || !widths || !w || !b || !ys)
    return fail(MJL_ERR_ARG, "small MLP: 1..%d layers of width 1..%d expected", kSmlMaxL, kSmlMaxW);
  std::memset(&P, 0, sizeof(P));
  P.nl = nl; P.k0 = k0;
  int wmax = fwd ? 1 : k0;
  for (int l = 0; l < nl; l++) {
    if (widths[l] < 1 || widths[l] > kSmlMaxW || !w[l] || !b[l] || !ys[l])
      return fail(MJL_ERR_ARG, "small MLP: layer %d: width 1..%d and non-null pointers expected", l, kSmlMaxW);
    P.n[l] = widths[l]; P.w[l] = w[l]; P.b[l] = b[l]; P.y[l] = ys[l];
    wmax = widths[l] > wmax ? widths[l] : wmax;
  }
  P.u = wmax <= 32 ? 32 : 64;
  return MJL_OK;
}

extern "C" int mjl_small_mlp_fwd(const float* x, int B, int k0, int nl, const int* widths, const float* const* w,
                                 const float* const* b, float* const* ys, void* stream) {
  SmallMlp P;
  int rc = small_mlp_setup(B, k0, nl, widths, w, b, ys, P, true);
  if (rc != MJL_OK) return rc;
  if (!x && B > 0) return fail(MJL_ERR_ARG, "bad argument");
  if (B == 0) return MJL_OK;
  const int R = kSmlThreads / P.u;
  hipLaunchKernelGGL(small_mlp_fwd_kernel<false>, dim3((unsigned)((B + R - 1) / R)), dim3(kSmlThreads), 0,
                     (hipStream_t)stream, x, B, P, ObsIn{});
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

extern "C" int mjl_small_mlp_bwd_input(const float* g_out, int B, int k0, int nl, const int* widths,
                                       const float* const* w, const float* const* ys, float* g_x, void* stream) {
  SmallMlp P;
  if (!w || !w[0]) return fail(MJL_ERR_ARG, "bad argument");
  const float* nob[kSmlMaxL] = {w[0], w[0], w[0], w[0]};  // biases unused by the backward
  int rc = small_mlp_setup(B, k0, nl, widths, w, nob, (float* const*)ys, P);
  if (rc != MJL_OK) return rc;
  if ((!g_out || !g_x) && B > 0) return fail(MJL_ERR_ARG, "bad argument");
  if (B == 0) return MJL_OK;
  const int R = kSmlThreads / P.u;
  hipLaunchKernelGGL(small_mlp_bwd_input_kernel<false>, dim3((unsigned)((B + R - 1) / R)), dim3(kSmlThreads), 0,
                     (hipStream_t)stream, g_out, B, P, g_x, ObsVjp{});
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

extern "C" int mjl_apg_obs(mjlBatch* B, const uint8_t* alive, const float* mean, const float* var, int use_norm,
                           float* o, float* on, uint8_t* alive_snap, void* stream) {
  if (!B || !alive || !o || !on || !alive_snap || (use_norm && (!mean || !var))) return fail(MJL_ERR_ARG, "bad argument");
  HIPCHK(hipSetDevice(B->device));
  const int nq = B->model->desc.nq, nv = B->model->desc.nv;
  const long n = (long)B->nenv * (nq + nv);
  hipLaunchKernelGGL(apg_obs_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, B->s,
                     B->nenv, nq, nv, alive, mean, var, use_norm, o, on, alive_snap);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

extern "C" int mjl_apg_post(mjlBatch* B, const float* rew, const float* term, const float* trunc, float gamma,
                            float diverge_qvel, uint8_t* alive, float* disc, float* ret, float* dropped, float* grew,
                            float* rfin, void* stream) {
  if (!B || !rew || !term || !trunc || !alive || !disc || !ret || !dropped || !grew || !rfin)
    return fail(MJL_ERR_ARG, "bad argument");
  HIPCHK(hipSetDevice(B->device));
  const ApgPostArgs a{gamma, diverge_qvel, alive, disc, ret, dropped, grew, rfin, B->nenv};
  hipLaunchKernelGGL(apg_post_kernel, dim3((B->nenv + kPostEnvs - 1) / kPostEnvs), dim3(64 * kPostEnvs), 0,
                     (hipStream_t)stream, B->s, B->model->desc.nq, B->model->desc.nv, rew, term, trunc, a);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

extern "C" int mjl_apg_obs_vjp(int B, int nq, int nv, const float* o, const uint8_t* alive_snap, const float* mean,
                               const float* var, int use_norm, const float* go, float* g_qpos, float* g_qvel,
                               void* stream) {
  if (B < 0 || nq < 0 || nv < 0 || !o || !alive_snap || !go || !g_qpos || !g_qvel || (use_norm && (!mean || !var)))
    return fail(MJL_ERR_ARG, "bad argument");
  const long n = (long)B * (nq + nv);
  if (n == 0) return MJL_OK;
  hipLaunchKernelGGL(apg_obs_vjp_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, B, nq,
                     nv, o, alive_snap, mean, var, use_norm, go, g_qpos, g_qvel);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

// mjl_apg_obs then mjl_small_mlp_fwd on its `on`, in one launch (k0 = nq + nv)
extern "C" int mjl_apg_obs_policy_fwd(mjlBatch* B, const uint8_t* alive, const float* mean, const float* var,
                                      int use_norm, float* o, float* on, uint8_t* alive_snap, int nl, const int* widths,
                                      const float* const* w, const float* const* b, float* const* ys, void* stream) {
  if (!B || !alive || !o || !on || !alive_snap || (use_norm && (!mean || !var))) return fail(MJL_ERR_ARG, "bad argument");
  const int nq = B->model->desc.nq, nv = B->model->desc.nv;
  SmallMlp P;
  int rc = small_mlp_setup(B->nenv, nq + nv, nl, widths, w, b, ys, P, true);
  if (rc != MJL_OK) return rc;
  HIPCHK(hipSetDevice(B->device));
  if (B->nenv == 0) return MJL_OK;
  const ObsIn O{B->s.qpos, B->s.qvel, nq, nv, use_norm, alive, mean, var, o, on, alive_snap};
  const int R = kSmlThreads / P.u;
  hipLaunchKernelGGL(small_mlp_fwd_kernel<true>, dim3((unsigned)((B->nenv + R - 1) / R)), dim3(kSmlThreads), 0,
                     (hipStream_t)stream, nullptr, B->nenv, P, O);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

// 1 if this batch's record launch is vjp_record_kernel (the rows in LDS; the post-step update and the next
// step's policy forward can ride along): the humanoid dims, rows not forced global
extern "C" int mjl_env_record_fused(const mjlBatch* B) {
  return B && B->model->nvc == 0 && !B->force_global_rows ? 1 : 0;
}

// the APG record + post-step update + the next step's observation and policy forward, in one launch
extern "C" int mjl_env_step_record_apg_next(mjlBatch* B, int slot, const float* act, float* obs, float* rew, float* term,
                                 float* trunc, float gamma, float diverge_qvel, uint8_t* alive, float* disc, float* ret,
                                 float* dropped, float* grew, float* rfin, const float* mean, const float* var,
                                 int use_norm, float* o, float* on, uint8_t* alive_snap, int nl, const int* widths,
                                 const float* const* w_t, const float* const* b, float* const* ys, void* stream) {
  if (!B || !act || !obs || !rew || !term || !trunc || !alive || !disc || !ret || !dropped || !grew || !rfin || !o ||
      !on || !alive_snap || (use_norm && (!mean || !var)))
    return fail(MJL_ERR_ARG, "bad argument");
  if (!B->has_env) return fail(MJL_ERR_ARG, "mjl_env_config not called");
  if (!B->d_vtape || slot < 0 || slot >= B->vtape_slots) return fail(MJL_ERR_ARG, "VJP tape slot %d not allocated", slot);
  if (!mjl_env_record_fused(B)) return fail(MJL_ERR_UNSUPPORTED, "record_apg_next: the humanoid dims' record only");
  const int nq = B->model->desc.nq, nv = B->model->desc.nv;
  SmallMlp P;
  int rc = small_mlp_setup(B->nenv, nq + nv, nl, widths, w_t, b, ys, P, true);
  if (rc != MJL_OK) return rc;
  KParams Pk = make_params(B);
  Pk.obs = obs; Pk.rew = rew; Pk.term = term; Pk.trunc = trunc;
  VjpArgs V;
  std::memset(&V, 0, sizeof(V));
  V.act = act;
  V.slot = B->d_vtape + (size_t)slot * B->nenv * (size_t)B->vtape_stride;
  V.post = ApgPostArgs{gamma, diverge_qvel, alive, disc, ret, dropped, grew, rfin, B->nenv};
  V.next = ApgNextArgs{use_norm, mean, var, o, on, alive_snap, P};
  return launch_vjp<true, 1>(B, V, stream, &Pk);
}

// the APG replay with the policy's input backward + the observation's backward added to its state
// cotangents, in one launch
extern "C" int mjl_env_step_vjp_replay_apg(mjlBatch* B, int slot, const float* act, const float* g_qpos,
                                           const float* g_qvel, const float* g_qacc_ws, const float* g_rew,
                                           const float* g_aux, float* out_qpos, float* out_qvel, float* out_qacc_ws,
                                           float* out_act, float* out_aux, float* nonfinite_count, int nl,
                                           const int* widths, const float* const* w, float* const* ys, const float* o,
                                           const uint8_t* alive_snap, const float* mean, const float* var,
                                           int use_norm, void* stream) {
  if (!B || !act || !g_qpos || !g_qvel || !g_rew || !g_aux || !out_qpos || !out_qvel || !out_act || !out_aux || !o ||
      !alive_snap || !w || !w[0] || (use_norm && (!mean || !var)))
    return fail(MJL_ERR_ARG, "bad argument");
  if (!B->has_env) return fail(MJL_ERR_ARG, "mjl_env_config not called");
  if (!B->d_vtape || slot < 0 || slot >= B->vtape_slots) return fail(MJL_ERR_ARG, "VJP tape slot %d not allocated", slot);
  const int nq = B->model->desc.nq, nv = B->model->desc.nv;
  SmallMlp Pm;
  const float* nob[kSmlMaxL] = {w[0], w[0], w[0], w[0]};  // biases unused by the backward
  int rc = small_mlp_setup(B->nenv, nq + nv, nl, widths, w, nob, ys, Pm);
  if (rc != MJL_OK) return rc;
  if (Pm.n[nl - 1] > 32 || B->model->desc.nu != Pm.n[nl - 1])
    return fail(MJL_ERR_ARG, "replay_apg: the policy's output width must be the action width (<= 32)");
  VjpArgs V;
  std::memset(&V, 0, sizeof(V));
  V.act = act; V.g_qpos = g_qpos; V.g_qvel = g_qvel; V.g_rew = g_rew; V.g_aux = g_aux;
  V.o_qpos = out_qpos; V.o_qvel = out_qvel; V.o_ctrl = out_act; V.o_aux = out_aux;
  V.g_ws = g_qacc_ws; V.o_ws = out_qacc_ws;
  V.nonfinite = nonfinite_count;
  V.slot = B->d_vtape + (size_t)slot * B->nenv * (size_t)B->vtape_stride;
  V.pbwd = ApgPolicyBwd{use_norm, o, mean, var, alive_snap, Pm};
  return launch_vjp<true, 2>(B, V, stream);
}

// mjl_small_mlp_bwd_input then mjl_apg_obs_vjp on its g_x, in one launch (k0 = nq + nv; g_x not stored)
extern "C" int mjl_apg_policy_bwd_obs_vjp(const float* g_out, int nenv, int nq, int nv, int nl, const int* widths,
                                          const float* const* w, const float* const* ys, const float* o,
                                          const uint8_t* alive_snap, const float* mean, const float* var, int use_norm,
                                          float* g_qpos, float* g_qvel, void* stream) {
  if (!w || !w[0]) return fail(MJL_ERR_ARG, "bad argument");
  if (nenv < 0 || nq < 0 || nv < 0 || ((!g_out || !o || !alive_snap || !g_qpos || !g_qvel) && nenv > 0) ||
      (use_norm && (!mean || !var)))
    return fail(MJL_ERR_ARG, "bad argument");
  SmallMlp P;
  const float* nob[kSmlMaxL] = {w[0], w[0], w[0], w[0]};  // biases unused by the backward
  int rc = small_mlp_setup(nenv, nq + nv, nl, widths, w, nob, (float* const*)ys, P);
  if (rc != MJL_OK) return rc;
  if (nenv == 0) return MJL_OK;
  const ObsVjp O{nq, nv, use_norm, o, alive_snap, mean, var, g_qpos, g_qvel};
  const int R = kSmlThreads / P.u;
  hipLaunchKernelGGL(small_mlp_bwd_input_kernel<true>, dim3((unsigned)((nenv + R - 1) / R)), dim3(kSmlThreads), 0,
                     (hipStream_t)stream, g_out, nenv, P, nullptr, O);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

// ---------------------------------------------------------------- PPO update losses
// rows per ppo_surrogate_kernel / twin_loss_head_kernel block (128: 0.2-0.3 ms per C5 per-rank
// update ahead of 64 and 256, profiles/r4/surrogate_rows_ab.txt)
constexpr int kSurrRows = 128;
extern "C" long long mjl_ppo_loss_scratch(int n, int A) {
  if (n <= 0 || A <= 0) return 0;
  const long long nb = (n + kLossT - 1) / kLossT, nbs = (n + kSurrRows - 1) / kSurrRows;
  return 3 * nb + nbs * (A + 1);
}

extern "C" int mjl_ppo_surrogate_clipped(const float* mean, const float* log_std, const float* act,
                                         const float* old_logp, const float* adv, const float* adv_stats,
                                         const int* stats_row, int n, int A, float clip_eps, float ent_coef,
                                         float log_std_lo, float log_std_hi, float* scratch, float* loss,
                                         float* g_mean, float* g_log_std, void* stream) {
  if (!mean || !log_std || !act || !old_logp || !adv || !scratch || !loss || !g_mean || !g_log_std || n <= 0 || A <= 0)
    return fail(MJL_ERR_ARG, "bad argument");
  if (A > kLossMaxA) return fail(MJL_ERR_UNSUPPORTED, "ppo surrogate: at most %d action columns", kLossMaxA);
  hipStream_t s = (hipStream_t)stream;
  const int nb_adv = (n + kLossT - 1) / kLossT, nb = (n + kSurrRows - 1) / kSurrRows;
  float* adv_part = scratch;
  float* part = scratch + 3 * (size_t)nb_adv;
  if (!adv_stats) hipLaunchKernelGGL(adv_stats_kernel, dim3(nb_adv), dim3(kLossT), 0, s, adv, n, adv_part);
  hipLaunchKernelGGL(ppo_surrogate_kernel<kSurrRows>, dim3(nb), dim3(kSurrRows), 0, s, mean, log_std, act, old_logp,
                     adv, n, A, clip_eps, adv_part, nb_adv, adv_stats, g_mean, part, log_std_lo, log_std_hi, stats_row);
  hipLaunchKernelGGL(ppo_surrogate_final_kernel, dim3(A + 1), dim3(64), 0, s, part, nb, n, A, log_std, ent_coef, loss,
                     g_log_std, log_std_lo, log_std_hi);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

extern "C" int mjl_ppo_surrogate(const float* mean, const float* log_std, const float* act, const float* old_logp,
                                 const float* adv, const float* adv_stats, int n, int A, float clip_eps,
                                 float ent_coef, float* scratch, float* loss, float* g_mean, float* g_log_std,
                                 void* stream) {
  return mjl_ppo_surrogate_clipped(mean, log_std, act, old_logp, adv, adv_stats, nullptr, n, A, clip_eps, ent_coef,
                                   -INFINITY, INFINITY, scratch, loss, g_mean, g_log_std, stream);
}

// rows per twin loss-head block: 64 at a data-parallel shard's minibatch (8,192 rows: 128 blocks where
// 128-row blocks left 192 of the 256 CUs idle), 128 at C3's 65,536
static int twin_loss_rows(int n) { return n <= 16384 ? 64 : kSurrRows; }
extern "C" long long mjl_twin_loss_head_blocks(int n) {
  return n > 0 ? (n + twin_loss_rows(n) - 1) / twin_loss_rows(n) : 0;
}

extern "C" int mjl_twin_loss_head(const float* z, const float* log_std, const float* act, const float* old_logp,
                                  const float* adv, const float* ret, const float* adv_stats, const int* stats_row,
                                  int n, int A, float clip_eps, float ent_coef, float log_std_lo, float log_std_hi,
                                  const float* bias, float* scratch, float* dz, float* lossp, float* glsp, float* biasp,
                                  void* stream) {
  if (!z || !log_std || !act || !old_logp || !adv || !ret || !scratch || !dz || !lossp || !glsp || !biasp || n <= 0 ||
      A <= 0)
    return fail(MJL_ERR_ARG, "bad argument");
  if (A > kLossMaxA || 2 * A + 2 > 64) return fail(MJL_ERR_UNSUPPORTED, "twin_loss_head: at most %d action columns", 31);
  hipStream_t s = (hipStream_t)stream;
  const int nb_adv = (n + kLossT - 1) / kLossT, nb = (int)mjl_twin_loss_head_blocks(n);
  if (!adv_stats) hipLaunchKernelGGL(adv_stats_kernel, dim3(nb_adv), dim3(kLossT), 0, s, adv, n, scratch);
  if (twin_loss_rows(n) == 64)
    hipLaunchKernelGGL(twin_loss_head_kernel<64>, dim3(nb), dim3(2 * 64), 0, s, z, log_std, act, old_logp, adv,
                       ret, n, A, clip_eps, ent_coef, scratch, nb_adv, adv_stats, stats_row, log_std_lo, log_std_hi, bias,
                       dz, lossp, glsp, biasp);
  else
    hipLaunchKernelGGL(twin_loss_head_kernel<kSurrRows>, dim3(nb), dim3(2 * kSurrRows), 0, s, z, log_std, act, old_logp,
                       adv, ret, n, A, clip_eps, ent_coef, scratch, nb_adv, adv_stats, stats_row, log_std_lo, log_std_hi,
                       bias, dz, lossp, glsp, biasp);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

// The twin update's fused thin ends (twin_kernels.hip). Shapes: bit 0 set when the gather + input
// layer launch has an instantiation for (k0, N), bit 1 when the output backward has one for (A, N),
// bit 2 when the fused head (forward + losses + backward) has one for (A, N = the last hidden width).
extern "C" int mjl_twin_fused_shapes(int k0, int A, int N) {
  return (k0 == kTinK0 && N == kTinN ? 1 : 0) | (A == kHbA && N > 0 && N % kHbCols == 0 ? 2 : 0) |
         (A == kThA && N == kThK ? 4 : 0);
}

// workgroups per net of the fused head launch (the partial rows of its reductions): 32-row chunks, two
// workgroups per CU (measured against 64-row chunks with one: 22.8 vs 27.7 us at 8,192 rows, 129.9 vs
// 179.6 us at 65,536; tools/twin_micro.hip)
extern "C" long long mjl_twin_head_blocks(int n) {
  if (n <= 0) return 0;
  const int nchunk = (n + kThRows - 1) / kThRows;
  return nchunk < kThBlocks / 2 ? nchunk : kThBlocks / 2;
}

extern "C" int mjl_twin_head(const float* zh, const float* bh, const float* W, const float* bo, const float* log_std,
                             const float* act, const float* old_logp, const float* adv, const float* ret,
                             const float* adv_stats, const int* stats_row, int n, int A, int K, float clip_eps,
                             float ent_coef, float log_std_lo, float log_std_hi, float* scratch, float* dzh, float* cs,
                             float* gw, float* lossp, float* glsp, float* biasp, void* stream) {
  if (!zh || !bh || !W || !bo || !log_std || !act || !old_logp || !adv || !ret || !dzh || !cs || !gw || !lossp ||
      !glsp || !biasp || n <= 0 || A <= 0 || K <= 0 || (!adv_stats && !scratch))
    return fail(MJL_ERR_ARG, "bad argument");
  if (!(mjl_twin_fused_shapes(0, A, K) & 4))
    return fail(MJL_ERR_UNSUPPORTED, "twin_head: %d outputs / hidden width %d not instantiated", A, K);
  if (n % kThRows) return fail(MJL_ERR_ARG, "twin_head: rows must be a multiple of %d", kThRows);
  if (((uintptr_t)zh | (uintptr_t)bh | (uintptr_t)W | (uintptr_t)dzh) % 16)
    return fail(MJL_ERR_ARG, "twin_head: 16-byte aligned zh, bh, W, dzh expected");
  hipStream_t s = (hipStream_t)stream;
  const int nb_adv = (n + kLossT - 1) / kLossT;
  if (!adv_stats) hipLaunchKernelGGL(adv_stats_kernel, dim3(nb_adv), dim3(kLossT), 0, s, adv, n, scratch);
  TwinHeadArgs p{zh, bh, W, bo, log_std, act, old_logp, adv, ret, adv_stats, stats_row, scratch, nb_adv, n, clip_eps,
                 ent_coef, log_std_lo, log_std_hi, dzh, cs, gw, lossp, glsp, biasp};
  hipLaunchKernelGGL((twin_head_kernel<kThA, kThK, kThRows>), dim3((unsigned)(2 * mjl_twin_head_blocks(n))), dim3(256), 0,
                     s, p);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

extern "C" int mjl_twin_gather_in(const long long* idx, const int* idx_row, int n, long long nsrc, int k0, int A,
                                  int N, const float* obs, const float* act, const float* logp, const float* ret,
                                  const float* adv, float* o2, float* a, float* ol, float* r, float* ad,
                                  const float* W, const float* b, float* h, void* stream) {
  if (!idx || !obs || !act || !logp || !ret || !adv || !o2 || !a || !ol || !r || !ad || !W || !b || !h || n <= 0 ||
      nsrc < 0 || A <= 0)
    return fail(MJL_ERR_ARG, "bad argument");
  if (!(mjl_twin_fused_shapes(k0, A, N) & 1))
    return fail(MJL_ERR_UNSUPPORTED, "twin_gather_in: input width %d / hidden width %d not instantiated", k0, N);
  if (((uintptr_t)h | (uintptr_t)b | (uintptr_t)W) % 16)
    return fail(MJL_ERR_ARG, "twin_gather_in: 16-byte aligned h, b and W expected");
  TwinInArgs p{idx, idx_row, n, A, nsrc, obs, act, logp, ret, adv, o2, a, ol, r, ad, W, b, h};
  const int nblk = 2 * ((n + kTinRows - 1) / kTinRows);  // a workgroup per (chunk, net), at most kTinBlocks
  hipLaunchKernelGGL((twin_gather_in_kernel<kTinK0, kTinN>), dim3((unsigned)(nblk < kTinBlocks ? nblk : kTinBlocks)),
                     dim3(kTinN), 0, (hipStream_t)stream, p);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

extern "C" int mjl_twin_head_bwd(const float* dz, const float* W, const float* y, int n, int A, int N, float* dzh,
                                 float* cs, float* gw, void* stream) {
  if (!dz || !W || !y || !dzh || !cs || !gw || n <= 0 || A <= 0 || N <= 0) return fail(MJL_ERR_ARG, "bad argument");
  if (!(mjl_twin_fused_shapes(0, A, N) & 2))
    return fail(MJL_ERR_UNSUPPORTED, "twin_head_bwd: %d outputs / hidden width %d not instantiated", A, N);
  if (n % kHbRows) return fail(MJL_ERR_ARG, "twin_head_bwd: rows must be a multiple of %d", kHbRows);
  if (((uintptr_t)W | (uintptr_t)y | (uintptr_t)dzh | (uintptr_t)cs | (uintptr_t)gw) % 16)
    return fail(MJL_ERR_ARG, "twin_head_bwd: 16-byte aligned buffers expected");
  TwinHeadBwdArgs p{dz, W, y, dzh, cs, gw, n, N};
  hipLaunchKernelGGL(twin_head_bwd_kernel<kHbA>, dim3((unsigned)(n / kHbRows), (unsigned)(N / kHbCols), 2), dim3(256),
                     0, (hipStream_t)stream, p);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

extern "C" int mjl_mse_strided(const float* v, int vstride, const float* r, int n, float* scratch, float* loss,
                               float* g_v, void* stream) {
  if (!v || !r || !scratch || !loss || !g_v || n <= 0 || vstride <= 0) return fail(MJL_ERR_ARG, "bad argument");
  hipStream_t s = (hipStream_t)stream;
  const int nb = (n + kLossT - 1) / kLossT;
  hipLaunchKernelGGL(mse_kernel, dim3(nb), dim3(kLossT), 0, s, v, vstride, r, n, g_v, scratch);
  hipLaunchKernelGGL(mse_final_kernel, dim3(1), dim3(64), 0, s, scratch, nb, n, loss);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

extern "C" int mjl_mse(const float* v, const float* r, int n, float* scratch, float* loss, float* g_v, void* stream) {
  return mjl_mse_strided(v, 1, r, n, scratch, loss, g_v, stream);
}

extern "C" int mjl_gather_rows_indexed(const long long* idx, const int* idx_row, int n, long long nsrc, int narr,
                                       const float* const* src, float* const* dst, const int* cols, void* stream) {
  if (!idx || n < 0 || nsrc < 0 || narr < 1 || narr > kGatherMax || !src || !dst || !cols)
    return fail(MJL_ERR_ARG, "bad argument");
  GatherArgs g;
  std::memset(&g, 0, sizeof(g));
  g.narr = narr;
  long long tot = 0;
  for (int k = 0; k < narr; k++) {
    if (!src[k] || !dst[k] || cols[k] <= 0) return fail(MJL_ERR_ARG, "bad argument");
    g.src[k] = src[k]; g.dst[k] = dst[k]; g.cols[k] = cols[k];
    tot += cols[k];
  }
  const long long work = (long long)n * tot;
  if (work == 0) return MJL_OK;
  if (work + 255 >= (1ll << 31)) return fail(MJL_ERR_ARG, "gather_rows: rows x total columns must be below 2^31");
  if (tot <= kGatherWaveCols) {
    GatherMap map;
    int q = 0;
    for (int k = 0; k < narr; k++)
      for (int c = 0; c < cols[k]; c++, q++) { map.k[q] = (unsigned char)k; map.c[q] = (unsigned char)c; }
    hipLaunchKernelGGL(gather_rows_wave_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, (hipStream_t)stream, idx,
                       n, nsrc, g, map, (int)tot, idx_row);
  } else {
    hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, (hipStream_t)stream, idx,
                       n, nsrc, g, idx_row);
  }
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

extern "C" int mjl_gather_rows(const long long* idx, int n, long long nsrc, int narr, const float* const* src,
                               float* const* dst, const int* cols, void* stream) {
  return mjl_gather_rows_indexed(idx, nullptr, n, nsrc, narr, src, dst, cols, stream);
}

static int adam_launch(int nt, float* const* p, const float* const* g, float* const* m, float* const* v,
                       const long long* numel, float lr, float beta1, float beta2, float eps, int step,
                       const float* step_dev, void* stream) {
  if (nt < 1 || nt > kAdamMaxT || !p || !g || !m || !v || !numel || (!step_dev && step < 1))
    return fail(MJL_ERR_ARG, "bad argument");
  AdamArgs a;
  std::memset(&a, 0, sizeof(a));
  a.nt = nt;
  for (int k = 0; k < nt; k++) {
    if (!p[k] || !m[k] || !v[k] || numel[k] < 0) return fail(MJL_ERR_ARG, "bad argument");
    a.p[k] = p[k]; a.g[k] = g[k]; a.m[k] = m[k]; a.v[k] = v[k];
    a.off[k + 1] = a.off[k] + numel[k];
  }
  if (!step_dev) {
    const float bc1 = 1.f - powf(beta1, (float)step), bc2 = 1.f - powf(beta2, (float)step);
    a.step_size = lr / bc1;
    a.bc2_sqrt = sqrtf(bc2);
  }
  a.step_dev = step_dev;
  a.lr = lr; a.b1 = beta1; a.b2 = beta2; a.eps = eps;
  const long long n = a.off[nt];
  if (n == 0) return MJL_OK;
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}

extern "C" int mjl_adam(int nt, float* const* p, const float* const* g, float* const* m, float* const* v,
                        const long long* numel, float lr, float beta1, float beta2, float eps, int step, void* stream) {
  return adam_launch(nt, p, g, m, v, numel, lr, beta1, beta2, eps, step, nullptr, stream);
}

extern "C" int mjl_adam_dev(int nt, float* const* p, const float* const* g, float* const* m, float* const* v,
                            const long long* numel, float lr, float beta1, float beta2, float eps, const float* step,
                            void* stream) {
  if (!step) return fail(MJL_ERR_ARG, "bad argument");
  return adam_launch(nt, p, g, m, v, numel, lr, beta1, beta2, eps, 0, step, stream);
}

extern "C" int mjl_adam_multi(int nt, float* const* p, const float* const* g, float* const* m, float* const* v,
                              const long long* numel, const int* group, int ngroups, const float* lr, float beta1,
                              float beta2, float eps, float gscale, float* const* step, int* ctr, int advanced,
                              void* stream) {
  if (nt < 1 || nt > kAdamMultiMaxT || ngroups < 1 || ngroups > kAdamMaxGroups || !p || !g || !m || !v || !numel ||
      !group || !lr || !step)
    return fail(MJL_ERR_ARG, "bad argument");
  AdamMultiArgs a;
  std::memset(&a, 0, sizeof(a));
  a.nt = nt; a.ngroups = ngroups;
  for (int k = 0; k < nt; k++) {
    if (!p[k] || !m[k] || !v[k] || numel[k] < 0 || group[k] < 0 || group[k] >= ngroups)
      return fail(MJL_ERR_ARG, "bad argument");
    a.p[k] = p[k]; a.g[k] = g[k]; a.m[k] = m[k]; a.v[k] = v[k]; a.grp[k] = group[k]; a.numel[k] = numel[k];
    const long long nb = (numel[k] + 255) / 256;
    if ((long long)a.blk[k] + nb >= (1LL << 30)) return fail(MJL_ERR_ARG, "adam_multi: too many elements");
    a.blk[k + 1] = a.blk[k] + (int)nb;
  }
  for (int gi = 0; gi < ngroups; gi++) {
    if (!step[gi]) return fail(MJL_ERR_ARG, "bad argument");
    for (int gj = 0; gj < gi; gj++)
      if (step[gj] == step[gi]) return fail(MJL_ERR_ARG, "adam_multi: groups need distinct step counters");
    a.lr[gi] = lr[gi]; a.step[gi] = step[gi];
  }
  a.b1 = beta1; a.b2 = beta2; a.eps = eps; a.gscale = gscale;
  a.tadd = advanced ? 0.f : 1.f;
  if (a.blk[nt] > 0)
    hipLaunchKernelGGL(adam_multi_kernel, dim3((unsigned)a.blk[nt]), dim3(256), 0, (hipStream_t)stream, a);
  if (!advanced)
    hipLaunchKernelGGL(step_counters_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, step[0],
                       ngroups > 1 ? step[1] : nullptr, ctr);
  HIPCHK(hipGetLastError());
  return MJL_OK;
}
