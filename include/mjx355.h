/*
 * mjx355 — MI355X-native batched humanoid physics step (C ABI).
 *
 * This header is the drop-in boundary for the reference's hot path. Each entry
 * point names the reference interface it replaces. The reference calls MJX, a JAX library
 * (mujoco-mjx==3.3.6, requirements.txt:27), from Python:
 *
 *   mujoco.MjModel.from_xml_path + mjx.put_model   src/training_utils.py:80,105
 *                                                  mjx_humanoid_speed_test.py:25,28,44
 *   mjx.make_data + mjx.forward                    src/envs.py:108-113 (single_pipeline_init)
 *   mjx.step                                       src/envs.py:345, mjx_humanoid_speed_test.py:54
 *   v_step = jit(vmap(single_step))                src/envs.py:333-495
 *   v_reset + merge_if_done (auto-reset)           src/envs.py:115-202,494; train_ppo.py:149-161
 *
 * Conventions
 *   - All device buffers are float32, C-contiguous, shape [nenv, dim] (one row per env).
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream). Calls are asynchronous.
 *   - Return value 0 = OK; otherwise an error code and mjl_last_error() holds a message.
 *   - A batch is thread-compatible, not thread-safe. One process per GPU.
 *   - No allocation happens in step/forward/env calls (they can be captured in a hipGraph).
 */
#ifndef MJX355_H_
#define MJX355_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------------------------------------
 * Model descriptor: compiled model constants (float64), the data that mjx.put_model uploads.
 * Filled by the host-side MJCF compiler (mjx_amd/mjcf.py). Capacities below bound the models
 * the kernels accept; larger models are rejected at load time (MJL_ERR_UNSUPPORTED).
 * ------------------------------------------------------------------------------------------- */
#define MJL_MAXBODY 32
#define MJL_MAXJNT 32
#define MJL_MAXQ 48
#define MJL_MAXV 32
#define MJL_MAXGEOM 32
#define MJL_MAXSITE 8
#define MJL_MAXU 32
#define MJL_MAXTENDON 4
#define MJL_MAXTENWRAP 4
#define MJL_MAXPAIR 256
#define MJL_MAXSENSOR 4
#define MJL_MAXOBS 64

/* enums (MuJoCo numbering where one exists) */
enum { MJL_GEOM_PLANE = 0, MJL_GEOM_SPHERE = 2, MJL_GEOM_CAPSULE = 3, MJL_GEOM_BOX = 6 };
enum { MJL_JNT_FREE = 0, MJL_JNT_HINGE = 3 };
enum { MJL_SOLVER_CG = 1, MJL_SOLVER_NEWTON = 2 };
enum { MJL_INT_EULER = 0, MJL_INT_IMPLICITFAST = 3 };
enum { MJL_COL_PLANE_SPHERE = 0, MJL_COL_PLANE_CAPSULE = 1, MJL_COL_SPHERE_SPHERE = 2,
       MJL_COL_SPHERE_CAPSULE = 3, MJL_COL_CAPSULE_CAPSULE = 4 };
enum { MJL_SENS_TOUCH = 0 };

typedef struct mjlModelDesc {
  int32_t nq, nv, nu, nbody, njnt, ngeom, nsite, ntendon, npair, nsensor, nsensordata;
  int32_t iterations, ls_iterations, solver, integrator, eulerdamp;
  double timestep, gravity[3], impratio, tolerance, ls_tolerance, meaninertia;

  int32_t body_parentid[MJL_MAXBODY], body_rootid[MJL_MAXBODY], body_weldid[MJL_MAXBODY];
  int32_t body_jntadr[MJL_MAXBODY], body_jntnum[MJL_MAXBODY];
  int32_t body_dofadr[MJL_MAXBODY], body_dofnum[MJL_MAXBODY];
  int32_t body_subtree_end[MJL_MAXBODY], body_level[MJL_MAXBODY];
  double body_pos[MJL_MAXBODY][3], body_quat[MJL_MAXBODY][4], body_ipos[MJL_MAXBODY][3];
  double body_inertia[MJL_MAXBODY][6]; /* body-frame tensor about ipos: xx yy zz xy xz yz */
  double body_mass[MJL_MAXBODY], body_invweight0[MJL_MAXBODY][2];

  int32_t jnt_type[MJL_MAXJNT], jnt_qposadr[MJL_MAXJNT], jnt_dofadr[MJL_MAXJNT];
  int32_t jnt_bodyid[MJL_MAXJNT], jnt_limited[MJL_MAXJNT];
  double jnt_pos[MJL_MAXJNT][3], jnt_axis[MJL_MAXJNT][3], jnt_range[MJL_MAXJNT][2];
  double jnt_stiffness[MJL_MAXJNT], jnt_margin[MJL_MAXJNT];
  double jnt_solref[MJL_MAXJNT][2], jnt_solimp[MJL_MAXJNT][5];

  int32_t dof_bodyid[MJL_MAXV], dof_jntid[MJL_MAXV], dof_parentid[MJL_MAXV];
  double dof_damping[MJL_MAXV], dof_armature[MJL_MAXV], dof_invweight0[MJL_MAXV];
  double qpos0[MJL_MAXQ], qpos_spring[MJL_MAXQ];

  int32_t geom_type[MJL_MAXGEOM], geom_bodyid[MJL_MAXGEOM];
  double geom_pos[MJL_MAXGEOM][3], geom_quat[MJL_MAXGEOM][4], geom_size[MJL_MAXGEOM][3];

  int32_t pair_geom1[MJL_MAXPAIR], pair_geom2[MJL_MAXPAIR], pair_kind[MJL_MAXPAIR];
  int32_t pair_condim[MJL_MAXPAIR];
  double pair_friction[MJL_MAXPAIR][5], pair_solref[MJL_MAXPAIR][2], pair_solimp[MJL_MAXPAIR][5];
  double pair_margin[MJL_MAXPAIR], pair_gap[MJL_MAXPAIR];

  int32_t site_type[MJL_MAXSITE], site_bodyid[MJL_MAXSITE];
  double site_pos[MJL_MAXSITE][3], site_quat[MJL_MAXSITE][4], site_size[MJL_MAXSITE][3];

  int32_t actuator_trnid[MJL_MAXU], actuator_ctrllimited[MJL_MAXU];
  double actuator_gear[MJL_MAXU], actuator_ctrlrange[MJL_MAXU][2];

  int32_t tendon_num[MJL_MAXTENDON], tendon_jnt[MJL_MAXTENDON][MJL_MAXTENWRAP];
  int32_t tendon_limited[MJL_MAXTENDON];
  double tendon_coef[MJL_MAXTENDON][MJL_MAXTENWRAP], tendon_range[MJL_MAXTENDON][2];
  double tendon_margin[MJL_MAXTENDON], tendon_solref[MJL_MAXTENDON][2];
  double tendon_solimp[MJL_MAXTENDON][5], tendon_invweight0[MJL_MAXTENDON];

  int32_t sensor_type[MJL_MAXSENSOR], sensor_objid[MJL_MAXSENSOR], sensor_adr[MJL_MAXSENSOR];
} mjlModelDesc;

/* Env configuration: EnvConfig (reference src/config.py:29-66) with the flip permutation
 * tables already expanded the way create_env_functions builds them (src/envs.py:48-74). */
typedef struct mjlEnvConfig {
  float progress_weight, electricity_cost, stall_torque_cost, posture_penalty_weight;
  float tall_height_threshold, tall_bonus_weight, target_threshold, target_dist;
  float stance_time_reward_weight, random_joint_noise, random_vel_noise, initial_velocity_max;
  float terminate_height, terminate_reward;
  int32_t stop_frames, max_episode_steps, random_flip;
  int32_t pelvis_body_id, head_body_id, touch_sensor_right_id, touch_sensor_left_id;
  int32_t obs_dim;
  int32_t act_perm[MJL_MAXU];
  float act_sign[MJL_MAXU];
  int32_t obs_perm[MJL_MAXOBS];
  float obs_sign[MJL_MAXOBS];
} mjlEnvConfig;

#define MJL_AUX_DIM 9 /* [flip, tx, ty, tz, close_count, stance, stance_time, last_pot, episode_step] */

/* error codes */
enum { MJL_OK = 0, MJL_ERR_ARG = 1, MJL_ERR_UNSUPPORTED = 2, MJL_ERR_HIP = 3, MJL_ERR_NOGPU = 4 };

/* readable per-env fields (mjl_get / mjl_set) */
enum {
  MJL_FIELD_QPOS = 0,          /* [nq]   Data.qpos */
  MJL_FIELD_QVEL = 1,          /* [nv]   Data.qvel */
  MJL_FIELD_QACC_WARMSTART = 2,/* [nv]   Data.qacc_warmstart */
  MJL_FIELD_TIME = 3,          /* [1]    Data.time */
  MJL_FIELD_CTRL = 4,          /* [nu]   Data.ctrl */
  MJL_FIELD_QACC = 5,          /* [nv]   Data.qacc (constrained forward acceleration) */
  MJL_FIELD_XPOS = 6,          /* [nbody*3] Data.xpos (from the last forward pass) */
  MJL_FIELD_XQUAT = 7,         /* [nbody*4] Data.xquat */
  MJL_FIELD_QFRC_ACTUATOR = 8, /* [nv]   Data.qfrc_actuator */
  MJL_FIELD_SENSORDATA = 9,    /* [nsensordata] Data.sensordata */
  MJL_FIELD_AUX = 10,          /* [9]    env aux state (src/envs.py:15) */
  MJL_FIELD_STATS = 11,        /* [4]    ncon_active, nefc_active, solver_iter, and nan_flag (env
                                          step) or the mean active rows per Newton Hessian (others) */
  MJL_FIELD_QFRC_BIAS = 12,    /* [nv]   Data.qfrc_bias */
  MJL_FIELD_QFRC_PASSIVE = 13, /* [nv]   Data.qfrc_passive */
  MJL_FIELD_QFRC_CONSTRAINT = 14, /* [nv] Data.qfrc_constraint */
  MJL_FIELD_QACC_SMOOTH = 15,  /* [nv]   Data.qacc_smooth */
  MJL_NFIELD = 16
};

typedef struct mjlModel mjlModel;
typedef struct mjlBatch mjlBatch;

/* Message of the last failing call on this thread. */
const char* mjl_last_error(void);
/* Library version string, "mjx355 <version> (gfx950) src=<hash>": <hash> is the sha256 prefix of the
   sources the library was built from (mjx_amd/_srchash.py); loaders compare it with their tree. */
const char* mjl_version(void);

/* Replaces mjx.put_model(MjModel) (src/training_utils.py:105): validate + upload constants.
 * Host only; does not need a GPU until mjl_batch_create. */
int mjl_model_create(const mjlModelDesc* desc, mjlModel** out);
void mjl_model_destroy(mjlModel* model);
/* Max constraint rows the model can produce (contacts + limits); sizes per-env scratch. */
int mjl_model_nefc_max(const mjlModel* model);

/* Replaces the batched mjx.make_data pytree (src/envs.py:110): owns per-env state on `device`,
 * initialised like make_data (qpos = qpos0, everything else zero). */
int mjl_batch_create(const mjlModel* model, int nenv, int device, mjlBatch** out);
void mjl_batch_destroy(mjlBatch* batch);
int mjl_batch_nenv(const mjlBatch* batch);

/* Batch options. MJL_OPT_STORE_DERIVED (default 1): step/env kernels also write the derived
 * per-env outputs (xpos, xquat, qacc, forces, sensordata, stats) readable with mjl_get; set 0 to
 * keep only the state + env outputs in the hot loop. MJL_OPT_FORCE_GLOBAL_ROWS (default 0, test
 * hook): keep constraint rows in the global-memory scratch even when they fit in LDS.
 * MJL_OPT_VJP_UNROLLED (default 0): the step VJPs differentiate the constraint solve's iterations
 * as executed (what jax.grad through MJX's fixed-count solver computes; reference train_apg.py:
 * 101-105,187-189 runs CG 4/4) instead of the implicit derivative at the converged active set; the
 * integrator's input is then qfrc_smooth + qfrc_constraint of the stopped solve. The VJP must see
 * the pre-step qacc_warmstart the forward step saw (the recompute replays that solve). Rejected for
 * models with iterations > 256 or ls_iterations > 31 (the tape's capacity); an env whose tape still
 * overflows gets NaN cotangents, or is cut and counted by the guarded VJPs.
 * MJL_OPT_VJP_TAPE (default 0): value = slots of the VJP tape (mjl_env_step_record /
 * mjl_env_step_vjp_replay), each holding one env step's forward workspace for every env
 * (~50 KB per env and slot for the humanoid; call outside stream capture; 0 frees it).
 * MJL_OPT_RESET_POOL (default 0): value = slots per env (<= 64) of the reset pool that
 * mjl_env_fill_reset_pool fills (call outside stream capture; 0 frees it). */
enum { MJL_OPT_STORE_DERIVED = 0, MJL_OPT_FORCE_GLOBAL_ROWS = 1, MJL_OPT_VJP_UNROLLED = 2, MJL_OPT_RESET_POOL = 3,
       MJL_OPT_VJP_TAPE = 4 };
int mjl_batch_set_option(mjlBatch* batch, int option, int value);

/* Copy a per-env field to / from a device buffer [nenv, dim] (async on stream). `mask` (device,
 * float [nenv], may be NULL) restricts mjl_set to envs with mask > 0.5. */
int mjl_get(mjlBatch* batch, int field, float* dst, void* stream);
int mjl_set(mjlBatch* batch, int field, const float* src, const float* mask, void* stream);

/* Replaces mjx.forward (src/envs.py:112): full forward pass, no integration, on envs with
 * mask > 0.5 (mask may be NULL = all). Results readable via mjl_get. */
int mjl_forward(mjlBatch* batch, const float* mask, void* stream);

/* Replaces mjx.step (src/envs.py:345): ctrl (device [nenv, nu], may be NULL = keep current)
 * -> forward + integrate, state updated in place. */
int mjl_step(mjlBatch* batch, const float* ctrl, void* stream);

/* Speed-test step (mjx_humanoid_speed_test.py:48-57): for each env e, a fresh make_data state
 * with qvel[0] = vel[e], one step, out[e] = new qpos[0]. Stateless: does not touch the batch
 * state (the batch only provides scratch and the model). */
int mjl_speedtest_step(mjlBatch* batch, const float* vel, float* out, void* stream);

/* Replaces create_env_functions' EnvConfig capture (src/envs.py:26-87). */
int mjl_env_config(mjlBatch* batch, const mjlEnvConfig* cfg);

/* Replaces v_step (src/envs.py:333-495) fused with the PPO auto-reset merge
 * (train_ppo.py:147-161): act [nenv, nu] -> obs [nenv, obs_dim], rew/term/trunc [nenv].
 * If auto_reset != 0, envs with max(term, trunc) > 0.5 are re-initialised in the same launch
 * (single_reset semantics, src/envs.py:115-202, RNG stream (seed, counter, env)) and obs holds
 * the post-reset observation, exactly as merge_if_done does; rew/term/trunc stay the step's. */
int mjl_env_step(mjlBatch* batch, const float* act, float* obs, float* rew, float* term,
                 float* trunc, int auto_reset, uint64_t seed, uint64_t counter, void* stream);

/* Reset pool: the v_reset half of train_ppo.py:147-161's merge_if_done, moved off the step's
 * critical path. A reset does not depend on the state it replaces, so resets can be computed in bulk
 * (full-occupancy launches) instead of one wave at a time at the end of a finishing env's step:
 * this fills slots 0..n-1 of every env (n = min(*dev_n, slots), device int read at execution
 * time), slot j drawn from (seed, (counter + j * 2^48) ^ 2^63, env) with the same single_reset semantics
 * (src/envs.py:115-202). Each later mjl_env_step(auto_reset=1) merges a finished env's next unused
 * slot; an env whose slots are used up resets in place from (seed, step counter, env) as before.
 * Requires MJL_OPT_RESET_POOL; not for key-drawn resets (mjl_env_set_reset_keys). */
int mjl_env_fill_reset_pool(mjlBatch* batch, const int* dev_n, uint64_t seed, uint64_t counter, void* stream);

/* RNG counter base for hipGraph capture of env steps / resets: if dev_counter_base (a device
 * uint64, may be NULL to detach) is set, the kernels draw with counter = the call's `counter` +
 * *dev_counter_base read at execution time, so a captured sequence of calls with counters 1..T
 * replays with fresh draws after the caller advances the base (src/envs.py:117 splits a fresh key
 * per reset; train_ppo.py:150 draws per rollout step). Eager callers leave it unset. */
int mjl_batch_set_counter_base(mjlBatch* batch, const uint64_t* dev_counter_base);

/* jax.random key modes: element i of a draw / split is threefry2x32(key, (0, i)) (jax >= 0.5
 * default, jax_threefry_partitionable; the reference pins jax==0.7.2, requirements.txt:17), or
 * the pre-0.5 layout (threefry over iota halves). */
enum { MJL_RNG_JAX_PARTITIONABLE = 1, MJL_RNG_JAX_ORIGINAL = 2 };

/* Replaces v_reset(keys) / merge_if_done's v_reset(random.split(key_reset, num_envs)) key input
 * (src/envs.py:116-147, train_ppo.py:150-152): if dev_keys (device uint32 [nenv, 2], read at
 * execution time; NULL detaches) is set, env resets — mjl_env_reset and the auto-reset of
 * mjl_env_step — draw from env e's jax.random key exactly as single_reset does (split(key, 4);
 * uniform(k1, (nq-7,)), uniform(k2, (nv,)), bernoulli(k3, .5), uniform(k4, (), 0, v_max)) instead of
 * (seed, counter): identical reset states to MJX for identical keys. */
int mjl_env_set_reset_keys(mjlBatch* batch, const uint32_t* dev_keys, int mode);

/* jax.random.split(key, num) for n keys at once: keys uint32 [n, 2] -> out [n, num, 2] (device). */
int mjl_prng_split(const uint32_t* keys, int n, int num, int mode, uint32_t* out, void* stream);

/* Replaces v_reset (src/envs.py:115-202,494) restricted to envs with mask > 0.5 (mask may be
 * NULL = all). obs [nenv, obs_dim] is written for reset envs only. `noise` (device, may be NULL)
 * overrides the on-device RNG with explicit draws [nenv, nq-7 + nv + 2] in [0,1):
 * joint-noise uniforms, velocity-noise uniforms, flip uniform, initial-speed uniform. */
int mjl_env_reset(mjlBatch* batch, const float* mask, uint64_t seed, uint64_t counter,
                  const float* noise, float* obs, void* stream);

/* Reverse-mode derivative of one mjl_step (APG backward; reference train_apg.py:161-209 takes
 * jax.value_and_grad through mjx.step, src/envs.py:345). The pre-step state is the batch state
 * (qpos, qvel, qacc_warmstart, ctrl), which is not modified. Given the cotangents of the step
 * outputs g_qpos [nenv,nq], g_qvel [nenv,nv], writes the cotangents of the inputs out_qpos
 * [nenv,nq], out_qvel [nenv,nv], out_ctrl [nenv,nu]. The constraint solve is differentiated at
 * its converged active set; qacc_warmstart gets no cotangent (DESIGN.md "APG"). */
int mjl_step_vjp(mjlBatch* batch, const float* g_qpos, const float* g_qvel, float* out_qpos,
                 float* out_qvel, float* out_ctrl, void* stream);

/* VJP of one env step (src/envs.py:333-492 single_step, without the reset merge) at the batch
 * state and aux with action act [nenv,nu]: cotangents of (qpos', qvel', reward, aux') ->
 * (qpos, qvel, action, aux). g_rew [nenv], g_aux / out_aux [nenv, MJL_AUX_DIM]. */
int mjl_env_step_vjp(mjlBatch* batch, const float* act, const float* g_qpos, const float* g_qvel,
                     const float* g_rew, const float* g_aux, float* out_qpos, float* out_qvel,
                     float* out_act, float* out_aux, void* stream);

/* Guarded env-step VJP for the APG reverse sweep: as mjl_env_step_vjp, but an env whose input
 * cotangents come out non-finite (a state blowing up inside the horizon) gets all-zero outputs and
 * increments *nonfinite_count (device float, may be NULL = unguarded). */
int mjl_env_step_vjp_guarded(mjlBatch* batch, const float* act, const float* g_qpos, const float* g_qvel,
                             const float* g_rew, const float* g_aux, float* out_qpos, float* out_qvel,
                             float* out_act, float* out_aux, float* nonfinite_count, void* stream);

/* Full-state VJPs: as mjl_step_vjp / mjl_env_step_vjp_guarded, plus the carried warm start.
 * g_qacc_ws [nenv,nv] is the cotangent of the output qacc_warmstart (= the step's qacc, MJX
 * solver.solve); out_qacc_ws [nenv,nv] receives the cotangent of the input qacc_warmstart, nonzero
 * only in MJL_OPT_VJP_UNROLLED mode when the truncated solve started from it (jax.grad through the
 * Data carry sees this path; a converged solve does not depend on its seed). Either may be NULL. */
int mjl_step_vjp_full(mjlBatch* batch, const float* g_qpos, const float* g_qvel, const float* g_qacc_ws,
                      float* out_qpos, float* out_qvel, float* out_qacc_ws, float* out_ctrl, void* stream);
int mjl_env_step_vjp_full(mjlBatch* batch, const float* act, const float* g_qpos, const float* g_qvel,
                          const float* g_qacc_ws, const float* g_rew, const float* g_aux, float* out_qpos,
                          float* out_qvel, float* out_qacc_ws, float* out_act, float* out_aux,
                          float* nonfinite_count, void* stream);

/* The persistent per-env state (what a step reads and writes: Data.qpos, qvel, qacc_warmstart,
 * time, plus the env aux) as packed rows [nenv, mjl_state_size] = [qpos | qvel | qacc_warmstart |
 * aux | time]: the APG remat tape entry (train_apg.py:187-189 checkpoints each step's carry).
 * mjl_set_state takes qacc_warmstart from ws_src (same row layout, may be NULL = from src). */
int mjl_state_size(const mjlBatch* batch);
int mjl_get_state(mjlBatch* batch, float* dst, void* stream);
int mjl_set_state(mjlBatch* batch, const float* src, const float* ws_src, void* stream);

/* Replaces compute_gae (train_ppo.py:171-202, a reverse lax.scan over the rollout): rew, term,
 * trunc [T, B], val [T+1, B] (val[T] = value of the obs after the last step) -> adv, ret [T, B],
 * delta = r + gamma V' (1 - term) - V, A = delta + gamma lam (1 - max(term, trunc)) A', ret = A + V.
 * Device pointers, float32, row-major; bit-identical to the elementwise formula (no contraction). */
int mjl_gae(const float* rew, const float* val, const float* term, const float* trunc, int T, int B,
            double gamma, double lam, float* adv, float* ret, void* stream);

/* The rollout step's elementwise work around the policy GEMMs (train_ppo.py:128-169), two launches
 * instead of the ~20 framework ops it takes as jnp / torch expressions:
 * mjl_obs_normalize replaces normalize_obs + clip (src/training_utils.py:52-56, train_ppo.py:134-135):
 *   y[n, dim] = clip((x - mean) / sqrt(var + 1e-8), -clip, clip).
 * mjl_policy_head replaces GaussianPolicy's tanh head + sampling + gaussian_logprob
 * (src/networks.py:82-112, train_ppo.py:121-126,136-139): z [B, A] = the MLP's last (linear) layer,
 *   mean = tanh(z), s = clip(log_std, -20, 2), act = mean + exp(s) eps, logp[B] = -0.5 sum((act -
 *   mean)^2 / exp(2 s) + 2 s + log 2 pi). Device pointers, float32, row-major. */
int mjl_obs_normalize(const float* x, const float* mean, const float* var, int n, int dim, float clip, float* y,
                      void* stream);
int mjl_policy_head(const float* z, const float* log_std, const float* eps, int B, int A, float* act, float* logp,
                    void* stream);

/* The rollout step's whole policy forward in one launch (train_ppo.py:134-139 with
 * src/networks.py:22-61,82-112: normalize_obs + clip, the GaussianPolicy MLP with tanh hidden
 * layers and a linear last layer, the tanh head, sampling and gaussian_logprob), on the matrix
 * cores: replaces mjl_obs_normalize + the MLP's GEMMs / activations + mjl_policy_head.
 * dims[0..nlayer] = obs_dim, hidden sizes..., act_dim (each <= 256, nlayer <= 6). params: per layer
 * WP[K/4][N][4] = W^T (K = in, N = out, both zero-padded to multiples of 16; WP[k/4][n][k%4] =
 * weight[n][k] of the torch / flax Dense) followed by the padded bias [N];
 * mjl_policy_param_floats(nlayer, dims) = its length. obs [B, obs_dim], eps [B, act_dim] -> act
 * [B, act_dim], logp [B]; device pointers, float32, row-major. */
long long mjl_policy_param_floats(int nlayer, const int* dims);
int mjl_policy_fwd(const float* obs, const float* mean, const float* var, float clip, const float* params, int nlayer,
                   const int* dims, const float* log_std, const float* eps, int B, float* act, float* logp,
                   void* stream);

/* APG with a stored forward instead of a recomputed one (train_apg.py:187-189 takes jax.grad with
 * per-step remat; HBM holds the forward instead): mjl_env_step_record is mjl_env_step without
 * auto-reset (same outputs and state update; derived fields are not stored) that also leaves in tape
 * slot `slot` what the step VJP's reverse passes read (workspace after integration, constraint rows,
 * the pre-step qpos / qvel / aux, the factor of the converged Hessian, the unrolled solve's tape);
 * mjl_env_step_vjp_replay is mjl_env_step_vjp_full of that step from the slot, without the
 * recompute and without restoring the pre-step state first. Requires MJL_OPT_VJP_TAPE; the VJP mode
 * (MJL_OPT_VJP_UNROLLED) must be the same at record and replay. On the humanoid dims the replay
 * (implicit, or unrolled with the CG solver) runs the lean layout: 19.5 KB of LDS per env, the dense
 * matrices read from the slot (environment MJL_VJP_LEAN=0 selects the full layout; same results). */
int mjl_env_step_record(mjlBatch* batch, int slot, const float* act, float* obs, float* rew, float* term,
                        float* trunc, void* stream);
/* mjl_env_step_record followed by mjl_apg_post's update of every env (below), as one launch where the
 * record keeps its rows in LDS (the implicit record on the humanoid dims), else the two launches. */
int mjl_env_step_record_apg(mjlBatch* batch, int slot, const float* act, float* obs, float* rew, float* term,
                            float* trunc, float gamma, float diverge_qvel, uint8_t* alive, float* disc, float* ret,
                            float* dropped, float* grew, float* rfin, void* stream);
/* 1 if mjl_env_step_record_apg_next applies to this batch (the implicit record on the humanoid dims). */
int mjl_env_record_fused(const mjlBatch* batch);
/* mjl_env_step_record_apg, then, from each env's new state and alive flag, mjl_apg_obs_policy_fwd's
 * observation (o, on, alive_snap) and small-MLP forward (ys) for the next rollout step, in the same
 * launch (the implicit record on the humanoid dims only: MJL_ERR_UNSUPPORTED otherwise). w_t[l]: layer
 * l's weight TRANSPOSED, [k_l, n_l] row-major; b[l], widths as mjl_small_mlp_fwd. */
int mjl_env_step_record_apg_next(mjlBatch* batch, int slot, const float* act, float* obs, float* rew, float* term,
                                 float* trunc, float gamma, float diverge_qvel, uint8_t* alive, float* disc, float* ret,
                                 float* dropped, float* grew, float* rfin, const float* mean, const float* var,
                                 int use_norm, float* o, float* on, uint8_t* alive_snap, int nl, const int* widths,
                                 const float* const* w_t, const float* const* b, float* const* ys, void* stream);
int mjl_env_step_vjp_replay(mjlBatch* batch, int slot, const float* act, const float* g_qpos, const float* g_qvel,
                            const float* g_qacc_ws, const float* g_rew, const float* g_aux, float* out_qpos,
                            float* out_qvel, float* out_qacc_ws, float* out_act, float* out_aux,
                            float* nonfinite_count, void* stream);
/* mjl_env_step_vjp_replay, then mjl_apg_policy_bwd_obs_vjp on its action cotangent, added to its state
 * cotangents before they are written (the same float operations), in one launch: w, widths, ys, o,
 * alive_snap, mean, var, use_norm as mjl_apg_policy_bwd_obs_vjp (the policy's output width = nu <= 32). */
int mjl_env_step_vjp_replay_apg(mjlBatch* batch, int slot, const float* act, const float* g_qpos,
                                const float* g_qvel, const float* g_qacc_ws, const float* g_rew, const float* g_aux,
                                float* out_qpos, float* out_qvel, float* out_qacc_ws, float* out_act, float* out_aux,
                                float* nonfinite_count, int nl, const int* widths, const float* const* w,
                                float* const* ys, const float* o, const uint8_t* alive_snap, const float* mean,
                                const float* var, int use_norm, void* stream);

/* APG rollout bookkeeping (train_apg.py:161-209; the sweep of mjx_amd/apg.py), one launch each per
 * rollout step. alive / alive_snap: uint8 [nenv] (0/1); device pointers, float32, row-major.
 * mjl_apg_obs: o [nenv, nq + nv] = [qpos | qvel] of each env (the APG observation); on = the policy
 *   input: x = alive ? o : 0, and with use_norm clip((x - mean) / (sqrt(var) + 1e-8), -10, 10)
 *   (train_apg.py:171-176); alive_snap = alive (for the backward).
 * mjl_apg_post: after the env step, per env: ok = rew, qpos, qvel finite (and max|qvel| <=
 *   diverge_qvel if > 0); bad = alive && !ok; dropped += bad; alive &= !bad; d = alive ? disc : 0;
 *   grew = -d / nenv (the reward's loss cotangent); ret += alive ? d rew : 0; rfin = rew if finite
 *   else 0; disc = d gamma (1 - max(term, trunc)); alive &= disc != 0.
 * mjl_apg_obs_vjp: g_qpos / g_qvel += (d on / d o)^T go at (o, alive_snap): zero where not alive,
 *   outside the clip, else go / (sqrt(var) + 1e-8) (go itself without use_norm). */
int mjl_apg_obs(mjlBatch* batch, const uint8_t* alive, const float* mean, const float* var, int use_norm, float* o,
                float* on, uint8_t* alive_snap, void* stream);
int mjl_apg_post(mjlBatch* batch, const float* rew, const float* term, const float* trunc, float gamma,
                 float diverge_qvel, uint8_t* alive, float* disc, float* ret, float* dropped, float* grew, float* rfin,
                 void* stream);
int mjl_apg_obs_vjp(int nenv, int nq, int nv, const float* o, const uint8_t* alive_snap, const float* mean,
                    const float* var, int use_norm, const float* go, float* g_qpos, float* g_qvel, void* stream);
/* The APG policy's per-step passes (src/networks.py:63-80 APGPolicy: Dense + tanh per layer, the
 * output tanh-squashed; train_apg.py:177 and its jax.grad): nl <= 4 layers, widths and k0 <= 64,
 * float32 row-major, w[l] = [widths[l], k_l] (torch Linear.weight), b[l] = [widths[l]], k_l = l ?
 * widths[l-1] : k0. mjl_small_mlp_fwd: ys[l] = tanh(ys[l-1] w[l]^T + b[l]) ([B, widths[l]], ys[-1] =
 * x), every sum in k order from the bias. mjl_small_mlp_bwd_input: g_x = d/dx of <g_out, ys[nl-1]>
 * from the forward's ys (the observation cotangent of the reverse sweep; no parameter gradients). */
int mjl_small_mlp_fwd(const float* x, int B, int k0, int nl, const int* widths, const float* const* w,
                      const float* const* b, float* const* ys, void* stream);
int mjl_small_mlp_bwd_input(const float* g_out, int B, int k0, int nl, const int* widths, const float* const* w,
                            const float* const* ys, float* g_x, void* stream);
/* The two fused per-step launches of the APG sweep (bit-identical to the pairs they replace):
 * mjl_apg_obs_policy_fwd = mjl_apg_obs, then mjl_small_mlp_fwd with x = on and k0 = nq + nv;
 * mjl_apg_policy_bwd_obs_vjp = mjl_small_mlp_bwd_input (k0 = nq + nv), then mjl_apg_obs_vjp with go = its
 * g_x (not stored). */
int mjl_apg_obs_policy_fwd(mjlBatch* batch, const uint8_t* alive, const float* mean, const float* var, int use_norm,
                           float* o, float* on, uint8_t* alive_snap, int nl, const int* widths, const float* const* w,
                           const float* const* b, float* const* ys, void* stream);
int mjl_apg_policy_bwd_obs_vjp(const float* g_out, int nenv, int nq, int nv, int nl, const int* widths,
                               const float* const* w, const float* const* ys, const float* o, const uint8_t* alive_snap,
                               const float* mean, const float* var, int use_norm, float* g_qpos, float* g_qvel,
                               void* stream);

/* PPO update (train_ppo.py:233-252, the bias-gradient column sums of every dense layer's backward
 * in value_and_grad of ppo_loss_fn / value_loss_fn, and the split-K weight-gradient sum):
 * out[d] = sum over rows of x[n, d] (row-major, float32, device), in a fixed order (two launches
 * when n > 256: per-chunk sums into `scratch`, then their sum). mjl_colsum_scratch(n, d) = the
 * scratch floats mjl_colsum needs (0: none, scratch may be NULL). */
long long mjl_colsum_scratch(int n, int d);
int mjl_colsum(const float* x, int n, int d, float* scratch, float* out, void* stream);
/* Backward of y = tanh(z) for a row-major [n, d] layer output (the PPO update's hidden layers; replaces
 * torch's tanh_backward + the bias gradient's column sum, src/networks.py:55-61 under jax.grad in
 * train_ppo.py:204-231): dz = g (1 - y^2), colsum_out[d] = dz.sum(0) in a fixed order (scratch: as
 * mjl_colsum). d % 4 == 0; g, y, dz, scratch and colsum_out 16-byte aligned. */
int mjl_tanh_bwd_colsum(const float* g, const float* y, int n, int d, float* dz, float* scratch, float* colsum_out,
                        void* stream);
/* out[e] = sum over s < ns of x[s * m + e] (slices summed in order: the split-K weight gradient's sum
 * over its batched GEMMs, in place of torch's sum(0)); m % 4 == 0, 16-byte aligned. */
int mjl_slice_sum(const float* x, int ns, long long m, float* out, void* stream);
/* x = tanh(x) elementwise in place (the update's hidden-layer activations, src/networks.py:55-61);
 * n % 4 == 0, 16-byte aligned. */
int mjl_tanh_inplace(float* x, long long n, void* stream);
/* The same reductions over nb stacked matrices (the twin update: the policy and value nets' layers
 * as one batched GEMM per layer, train_ppo.py:233-252 taking both nets' steps per minibatch):
 * x [nb][n][d] -> out [nb][d], each matrix summed in mjl_colsum's order; for nb > 1, n must be a
 * multiple of the 128-row chunk (n > 256). scratch: mjl_colsum_batched_scratch(nb, n, d) floats.
 * mjl_slice_sum_batched: out[b][e] = sum over s < ns of x[(b * ns + s) * m + e]. */
long long mjl_colsum_batched_scratch(int nb, int n, int d);
/* The first stage alone, with the caller's row chunk: dz = g (1 - y^2) written out and partials
 * [nb][n / chunk][d] = each chunk's column sums of dz, for mjl_slice_sum_multi to finish.
 * n % chunk == 0, d % 4 == 0, 16-byte aligned buffers. */
int mjl_tanh_bwd_colsum_partials(const float* g, const float* y, int nb, int n, int d, int chunk, float* dz,
                                 float* partials, void* stream);
int mjl_colsum_batched(const float* x, int nb, int n, int d, float* scratch, float* out, void* stream);
int mjl_tanh_bwd_colsum_batched(const float* g, const float* y, int nb, int n, int d, float* dz, float* scratch,
                                float* colsum_out, void* stream);
int mjl_slice_sum_batched(const float* x, int nb, int ns, long long m, float* out, void* stream);
/* nseg <= 16 slice sums in one launch: out_k[b][e] = sum over s < ns[k] (in order) of
 * x_k[(b * ns[k] + s) * m[k] + e], b < nb[k] (the twin update's weight-gradient slices and column-sum
 * partials of every layer, reduced together at the end of its backward). step0 / step1 / ctr (device
 * float / float / int, each or NULL) are advanced by one in the same launch: the captured update's
 * step counters and minibatch row, after their last read in the step (mjl_adam_multi then runs with
 * advanced = 1). */
int mjl_slice_sum_multi(int nseg, const float* const* x, float* const* out, const int* nb, const int* ns,
                        const long long* m, float* step0, float* step1, int* ctr, void* stream);
/* The twin update's losses and output-layer backward in one pass (train_ppo.py:204-220 for both nets):
 * z [2][n][A], z[0] = the policy's mean (tanh of its last Dense, networks.py:103), z[1][:, 0] = the
 * value (the value net's output layer padded to A rows); the clipped surrogate as
 * mjl_ppo_surrogate_clipped (advantages normalised by adv_stats — a [n_minibatches, 2] table read at
 * *stats_row when stats_row is given — or over the n rows when adv_stats is NULL), the value loss
 * mean (v - ret)^2 (train_ppo.py:218-220). Writes dz [2][n][A]: dz[0] = d loss / d mean (1 - mean^2),
 * dz[1][:, 0] = 2 (v - ret) / n, dz[1][:, 1:] = 0; and per block b < mjl_twin_loss_head_blocks(n) the
 * partials whose in-order sums over b (mjl_slice_sum_multi) are the results: lossp [nb] -> the policy
 * loss, glsp [nb][A] -> d loss / d log_std (clip mask included), biasp [2][nb][A] -> both output
 * biases' gradients. bias (or NULL): z holds the output layers' pre-activations and bias [2][A] their
 * biases — mean = tanh(z[0] + bias[0]), v = z[1][:, 0] + bias[1][0]. scratch: mjl_ppo_loss_scratch(n, A)
 * floats. A <= 32. */
long long mjl_twin_loss_head_blocks(int n);

/* The twin PPO update's thin ends as single launches (train_ppo.py:233-252 run_ppo_updates over the
   src/networks.py:82-131 MLPs; both nets stacked as in mjl_twin_loss_head). Bit 0 of
   mjl_twin_fused_shapes: mjl_twin_gather_in is instantiated for (k0, N); bit 1: mjl_twin_head_bwd for
   (A, N). Other shapes take the library GEMM path. */
int mjl_twin_fused_shapes(int k0, int A, int N);
/* The minibatch gather (make_index_batches' rows, train_ppo.py:222-231; idx [n], or row *idx_row of an
   [n_minibatches, n] table) fused with both nets' input layer: o2 [2, n, k0] (the observations twice),
   a [n, A], ol / r / ad [n] gathered from obs / act / logp / ret / adv (an out-of-range index gives NaN);
   h [2, n, N] = tanh(o W[net]^T + b[net]) with W [2, N, k0], b [2, N]. */
int mjl_twin_gather_in(const long long* idx, const int* idx_row, int n, long long nsrc, int k0, int A, int N,
                       const float* obs, const float* act, const float* logp, const float* ret, const float* adv,
                       float* o2, float* a, float* ol, float* r, float* ad, const float* W, const float* b,
                       float* h, void* stream);
/* The output layers' backward fused with the last hidden layer's tanh backward: dzh [2, n, N] =
   (dz W) (1 - y^2) for dz [2, n, A], W [2, A, N], y [2, n, N]; per chunk c of 128 rows the column sums of
   dzh into cs [2, n/128, N] and the output weight gradient's partial dz^T y into gw [2, n/128, A, N]
   (summed by mjl_slice_sum_multi). n % 128 == 0, 16-byte aligned buffers. */
int mjl_twin_head_bwd(const float* dz, const float* W, const float* y, int n, int A, int N, float* dzh, float* cs,
                      float* gw, void* stream);
/* The twin update's whole head in one launch (bit 2 of mjl_twin_fused_shapes; train_ppo.py:204-220 on
   both nets' output layers): H = tanh(zh + bh) for the last hidden layer's bias-less GEMM output zh
   [2, n, K] and bias bh [2, K]; z = H W^T + bo (W [2, A, K], bo [2, A]); the policy's clipped
   surrogate + entropy and the value's MSE gradient exactly as mjl_twin_loss_head (advantages
   normalised by row *stats_row of adv_stats, or, adv_stats NULL, by this minibatch's own statistics
   through scratch of mjl_ppo_loss_scratch(n, A) floats); then dzh [2, n, K] = (dz W)(1 - H^2). Per
   workgroup b < S = mjl_twin_head_blocks(n) of each net k, partials summed in order by
   mjl_slice_sum_multi: lossp[b] (policy loss, b = 0 adds the entropy term), glsp[b][A] (log_std),
   biasp[k][b][A] (output biases), cs[k][b][K] (the last hidden bias), gw[k][b][A][K] (output weights).
   n % 64 == 0. */
long long mjl_twin_head_blocks(int n);
int mjl_twin_head(const float* zh, const float* bh, const float* W, const float* bo, const float* log_std,
                  const float* act, const float* old_logp, const float* adv, const float* ret, const float* adv_stats,
                  const int* stats_row, int n, int A, int K, float clip_eps, float ent_coef, float log_std_lo,
                  float log_std_hi, float* scratch, float* dzh, float* cs, float* gw, float* lossp, float* glsp,
                  float* biasp, void* stream);
int mjl_twin_loss_head(const float* z, const float* log_std, const float* act, const float* old_logp, const float* adv,
                       const float* ret, const float* adv_stats, const int* stats_row, int n, int A, float clip_eps,
                       float ent_coef, float log_std_lo, float log_std_hi, const float* bias, float* scratch,
                       float* dz, float* lossp, float* glsp, float* biasp, void* stream);
/* x[b][r][j] = act_b(x[b][r][j] + bias[b][j]) in place over nb stacked row-major [rows, n] matrices,
 * act_b = tanh when bit b of act_mask is set, else the identity (the twin update's dense-layer
 * epilogue, src/networks.py:55-61, after a bias-less batched GEMM). */
int mjl_bias_act(float* x, const float* bias, int nb, long long rows, int n, unsigned act_mask, void* stream);

/* PPO update losses (train_ppo.py:204-220), forward and gradient in one pass, deterministic.
 * mjl_ppo_surrogate: loss = -mean_i min(r_i an_i, clip(r_i, 1 - clip_eps, 1 + clip_eps) an_i)
 *   - ent_coef 0.5 sum_j (1 + log 2 pi + 2 log_std_j) / A, with r_i = exp(logp_i - old_logp_i),
 *   logp the diagonal Gaussian log-density of act under (mean, exp(log_std)) and an the advantage
 *   normalised over the n rows, (adv - mean) / (population std + 1e-8) — or by adv_stats = (mean,
 *   std) when given (device, the data-parallel minibatch's global statistics); g_mean [n, A] and
 *   g_log_std [A] are d loss / d mean and d loss / d log_std (torch.minimum / clamp conventions for
 *   ties and bounds). mjl_mse: loss = mean (v - r)^2, g_v = 2 (v - r) / n. scratch:
 *   mjl_ppo_loss_scratch(n, A) floats (mjl_mse needs n / 256 + 1). A <= 32.
 * mjl_gather_rows: dst_k[r, :] = src_k[idx[r], :] for narr <= 8 row-major float arrays of nsrc rows
 *   and cols[k] columns (the minibatch gather of train_ppo.py:237-241), idx int64 [n]; one launch;
 *   an index outside [0, nsrc) gives a NaN row; n x (total columns) must be below 2^31. */
long long mjl_ppo_loss_scratch(int n, int A);
int mjl_ppo_surrogate(const float* mean, const float* log_std, const float* act, const float* old_logp,
                      const float* adv, const float* adv_stats, int n, int A, float clip_eps, float ent_coef,
                      float* scratch, float* loss, float* g_mean, float* g_log_std, void* stream);
int mjl_mse(const float* v, const float* r, int n, float* scratch, float* loss, float* g_v, void* stream);
/* mjl_ppo_surrogate with log_std clipped to [log_std_lo, log_std_hi] on read (networks.py:103 clips it
 * to [-20, 2]) and g_log_std zero where the raw value lies outside (torch.clamp's backward, bounds
 * inclusive); +-INFINITY bounds = mjl_ppo_surrogate. stats_row (device int, or NULL): adv_stats is an
 * [n_minibatches, 2] table read at that row (a captured minibatch step reads its row at run time). */
int mjl_ppo_surrogate_clipped(const float* mean, const float* log_std, const float* act, const float* old_logp,
                              const float* adv, const float* adv_stats, const int* stats_row, int n, int A,
                              float clip_eps, float ent_coef, float log_std_lo, float log_std_hi, float* scratch,
                              float* loss, float* g_mean, float* g_log_std, void* stream);
/* mjl_mse with v[i] read at v + i * vstride (the value column of the twin update's padded output). */
int mjl_mse_strided(const float* v, int vstride, const float* r, int n, float* scratch, float* loss, float* g_v,
                    void* stream);
int mjl_gather_rows(const long long* idx, int n, long long nsrc, int narr, const float* const* src, float* const* dst,
                    const int* cols, void* stream);
/* mjl_gather_rows from row *idx_row (device int) of an [n_minibatches, n] index table (NULL: idx). */
int mjl_gather_rows_indexed(const long long* idx, const int* idx_row, int n, long long nsrc, int narr,
                            const float* const* src, float* const* dst, const int* cols, void* stream);
/* Adam (optax.adam defaults as train_ppo.py:84-85 build them; torch.optim.Adam's fused update) over
 * nt <= 16 float32 tensors in one launch: m = b1 m + (1 - b1) g, v = b2 v + (1 - b2) g^2,
 * p -= lr / (1 - b1^step) m / (sqrt(v) / sqrt(1 - b2^step) + eps); g[k] NULL skips tensor k. */
int mjl_adam(int nt, float* const* p, const float* const* g, float* const* m, float* const* v,
             const long long* numel, float lr, float beta1, float beta2, float eps, int step, void* stream);
/* mjl_adam with the step count read from device memory at execution time (step: device float, the
 * step being taken, >= 1), so a hipGraph that captured the call takes the bias corrections of each
 * replay's own step (the caller's captured increment advances it; train_ppo.py:233-252 runs the whole
 * update as one compiled scan, optax keeping the count as device state). */
int mjl_adam_dev(int nt, float* const* p, const float* const* g, float* const* m, float* const* v,
                 const long long* numel, float lr, float beta1, float beta2, float eps, const float* step,
                 void* stream);

/* Adam over nt <= 24 tensors of up to 2 optimisers in one launch (the PPO update's policy and value
 * steps, train_ppo.py:246-251): tensor k uses group[k]'s lr and device step counter step[group[k]]
 * (float, the count before this step: the step takes step + 1, and every group's counter is advanced
 * by one after it); g is scaled by gscale (the data-parallel mean: 1 / world size); ctr (device int,
 * or NULL) is advanced with the counters. advanced = 1: the counters were advanced earlier in the
 * minibatch step (mjl_slice_sum_multi's step0 / step1 / ctr): the step takes step as it is and
 * nothing is advanced here. Same arithmetic as mjl_adam_dev. */
int mjl_adam_multi(int nt, float* const* p, const float* const* g, float* const* m, float* const* v,
                   const long long* numel, const int* group, int ngroups, const float* lr, float beta1, float beta2,
                   float eps, float gscale, float* const* step, int* ctr, int advanced, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MJX355_H_ */
