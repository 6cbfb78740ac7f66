// Device-side model constants (float32) and kernel parameter block.
// Built on the host from mjlModelDesc (include/mjx355.h) by mjl_model_create; lives in device
// global memory, read through the scalar/vector caches (a few KB, shared by every env).
#pragma once
#include <stdint.h>

#include "../../include/mjx355.h"

namespace mjl {

// Packed per-lane records (16-byte rows -> one b128 load each): a phase loads the records of
// its lane once, up front, instead of walking dependent index chains inside its level loops.
struct alignas(16) BodyRec {
  int parent, level, jntadr, jntnum;
  int dofadr, dofnum, subtree_end, rootid;
  int isfree, qadr, pad0, pad1;  // isfree: the body's only joint is free (qadr: its qpos address)
  float pos[3], mass;
  float quat[4];
  float ipos[3], pad2;
  float inertia[6], pad3[2];  // body_inertia (local principal frame: xx yy zz xy xz yz)
};
// the first three hinges of a body (kinematics' local transform), by body: one load with the body's
// own record instead of a second load through jntadr
struct alignas(16) HingeRec {
  float pos[3], pad0;
  float axis[3], pad1;
};
// geom (index < 32) / site (index 32 + s) frame constants, by lane: body, local pos, local z axis
// (geoms, mat[0..2]) or local rotation (sites)
struct alignas(16) FrameRec {
  int body, pad0, pad1, pad2;
  float pos[3], pad3;
  float mat[9], pad4[3];
};
struct alignas(16) JntRec {  // hinge joints (local frame of the body)
  float pos[3], qpos0;
  float axis[3];
  int qadr;
  int body, parent, isfree, dofadr;
};
struct alignas(16) DofRec {
  int bodyid, jntid, rootid, kfree;  // kfree: index 0..5 inside a free joint, -1 otherwise
  uint32_t ancmask;                  // bit j set <=> dof j is this dof or one of its ancestors
  int qadr_spring;                   // qpos address of a hinge spring, -1 when none
  float damping, armature;
  float stiffness, qpos_spring, invweight0, pad;
};
struct alignas(16) PairRec {
  int g1, g2, kind, condim;
  float r1, h1, r2, h2;  // geom_size[:, 0:2] of both geoms
  float includemargin, mu, invweight, pad;
  uint32_t mask1, mask2;  // body_dofmask of both bodies
  int b1, b2;
};
// a limit-row candidate: lane = joint (limited hinge) or lane = tendon (limited tendon); everything
// the row needs, including its impedance parameters, in one record
struct alignas(16) LimRec {
  int on, qadr, dofadr, pad;  // on: the joint / tendon is a limit-row candidate
  float lo, hi, margin, invweight;
  float solref[2], solimp[5], pad1;
};

struct ModelF {
  int nq, nv, nu, nbody, njnt, ngeom, nsite, ntendon, npair, nsensor, nsensordata;
  int iterations, ls_iterations, solver, integrator, eulerdamp, maxlevel, nlimited, any_damping;
  int nroot, root[MJL_MAXBODY];  // kinematic roots: bodies whose parent is the world
  float timestep, gravity[3], impratio, tolerance, ls_tolerance, meaninertia, scale;

  int body_parentid[MJL_MAXBODY], body_rootid[MJL_MAXBODY], body_jntadr[MJL_MAXBODY];
  int body_jntnum[MJL_MAXBODY], body_dofadr[MJL_MAXBODY], body_dofnum[MJL_MAXBODY];
  int body_subtree_end[MJL_MAXBODY], body_level[MJL_MAXBODY];
  uint32_t body_dofmask[MJL_MAXBODY];  // bit d set <=> dof d moves body b (ancestor chain)
  // tree walks of the reverse passes as bit loops (no record loads in the loop): ancestors-or-self
  // (world excluded), children, children without a free joint, joints whose world anchor / axis
  // cotangents gather into b (b's free joint, hinges of b's children); the float sum of the masses
  // of root r's subtree in body order
  uint32_t body_ancmask[MJL_MAXBODY], body_childmask[MJL_MAXBODY], body_childmask_nf[MJL_MAXBODY];
  uint32_t body_jgather[MJL_MAXBODY];
  uint32_t dof_descmask[MJL_MAXV];  // bit i set <=> dof i is this dof or one of its descendants
  uint32_t body_geommask[MJL_MAXBODY];  // bit g set <=> geom g belongs to body b
  float body_rootmass[MJL_MAXBODY];
  float body_pos[MJL_MAXBODY][3], body_quat[MJL_MAXBODY][4], body_ipos[MJL_MAXBODY][3];
  float body_inertia[MJL_MAXBODY][6], body_mass[MJL_MAXBODY], body_invweight0[MJL_MAXBODY][2];

  int jnt_type[MJL_MAXJNT], jnt_qposadr[MJL_MAXJNT], jnt_dofadr[MJL_MAXJNT], jnt_limited[MJL_MAXJNT];
  float jnt_pos[MJL_MAXJNT][3], jnt_axis[MJL_MAXJNT][3], jnt_range[MJL_MAXJNT][2];
  float jnt_stiffness[MJL_MAXJNT], jnt_margin[MJL_MAXJNT], jnt_solref[MJL_MAXJNT][2];
  float jnt_solimp[MJL_MAXJNT][5];

  int dof_bodyid[MJL_MAXV], dof_jntid[MJL_MAXV], dof_parentid[MJL_MAXV];
  float dof_damping[MJL_MAXV], dof_armature[MJL_MAXV], dof_invweight0[MJL_MAXV];
  float qpos0[MJL_MAXQ], qpos_spring[MJL_MAXQ];

  int geom_type[MJL_MAXGEOM], geom_bodyid[MJL_MAXGEOM];
  float geom_pos[MJL_MAXGEOM][3], geom_zaxis[MJL_MAXGEOM][3], geom_size[MJL_MAXGEOM][3];

  int pair_geom1[MJL_MAXPAIR], pair_geom2[MJL_MAXPAIR], pair_kind[MJL_MAXPAIR], pair_condim[MJL_MAXPAIR];
  float pair_mu[MJL_MAXPAIR], pair_solref[MJL_MAXPAIR][2], pair_solimp[MJL_MAXPAIR][5];
  float pair_includemargin[MJL_MAXPAIR], pair_invweight[MJL_MAXPAIR];  // invweight incl. pyramid factor

  int site_bodyid[MJL_MAXSITE];
  float site_pos[MJL_MAXSITE][3], site_mat[MJL_MAXSITE][9], site_size[MJL_MAXSITE][3];

  int actuator_dof[MJL_MAXU], actuator_ctrllimited[MJL_MAXU];
  float actuator_gear[MJL_MAXU], actuator_ctrlrange[MJL_MAXU][2];

  int tendon_num[MJL_MAXTENDON], tendon_qadr[MJL_MAXTENDON][MJL_MAXTENWRAP];
  int tendon_dof[MJL_MAXTENDON][MJL_MAXTENWRAP], tendon_limited[MJL_MAXTENDON];
  float tendon_coef[MJL_MAXTENDON][MJL_MAXTENWRAP], tendon_range[MJL_MAXTENDON][2];
  float tendon_margin[MJL_MAXTENDON], tendon_solref[MJL_MAXTENDON][2], tendon_solimp[MJL_MAXTENDON][5];
  float tendon_invweight0[MJL_MAXTENDON];

  int sensor_type[MJL_MAXSENSOR], sensor_objid[MJL_MAXSENSOR], sensor_adr[MJL_MAXSENSOR];

  BodyRec brec[MJL_MAXBODY];
  JntRec jrec[MJL_MAXJNT];
  DofRec drec[MJL_MAXV];
  PairRec prec[MJL_MAXPAIR];
  LimRec jlim[MJL_MAXJNT], tlim[MJL_MAXTENDON];
  HingeRec bhinge[MJL_MAXBODY][3];
  FrameRec frec[64];
};

enum Mode { MODE_FORWARD = 0, MODE_STEP = 1, MODE_SPEEDTEST = 2, MODE_ENV_STEP = 3, MODE_ENV_RESET = 4 };

// per-env state rows, [nenv, dim] each
struct StateBuf {
  float *qpos, *qvel, *qacc_warmstart, *time, *ctrl, *aux;
  // derived (outputs of the last forward pass)
  float *qacc, *xpos, *xquat, *qfrc_actuator, *sensordata, *stats;
  float *qfrc_bias, *qfrc_passive, *qfrc_constraint, *qacc_smooth;
};

struct KParams {
  const ModelF* m;
  const mjlEnvConfig* env;
  StateBuf s;
  int nenv;
  int store_derived;
  int force_global_rows;  // test hook: always use the global-scratch row storage
  int auto_reset;
  const float* in_ctrl;   // [nenv, nu] or null
  const float* mask;      // [nenv] or null
  const float* noise;     // [nenv, nq-7+nv+2] or null
  const float* vel;       // speed test input
  float* out_speed;       // speed test output
  float *obs, *rew, *term, *trunc;
  float* scratch;         // global overflow rows, [nenv, scratch_stride]
  int scratch_stride;    // floats per env
  int gmax_efc, gmax_con; // row / contact capacity of one scratch slab
  uint32_t seed_lo, seed_hi, ctr_lo, ctr_hi;
  const unsigned long long* ctr_base;  // device counter base added to (ctr_hi, ctr_lo), or null
  const uint32_t* keys;                // per-env jax.random reset keys [nenv, 2], or null
  int key_mode;                        // MJL_RNG_* of `keys`
  // reset pool (mjl_env_fill_reset_pool): slot j of env e is row j * nenv + e of `rs` / rs_obs
  StateBuf rs;
  float* rs_obs;    // [slots * nenv, obs_dim]
  int* pool_ctl;    // [nenv, 2]: next unused slot, filled slots; null = no pool
  const int* pool_n;  // fill: slots to fill (device int, read at execution time)
  int pool_slot;    // fill: the slot this launch draws (-1: not a fill)
  int pool_slots;   // fill: pool capacity (slots per env)
};

}  // namespace mjl
