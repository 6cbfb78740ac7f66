// ORACLE — TEST INFRASTRUCTURE ONLY (see physics.hpp header).
//
// Serial restatement of the reference env wrapper around mjx.step:
//   single_reset  reference src/envs.py:115-202 (random pose/vel, 2x forward, target, aux, obs)
//   single_step   reference src/envs.py:333-492 (flip, clip, step, reward, aux, obs, term/trunc)
//   compute_obs   reference src/envs.py:317-331 ; get_body_velocities_local :274-315
//   get_stance    reference src/envs.py:89-106
// The random draws are inputs here (explicit uniforms), so the product's RNG is tested separately.
#pragma once
#include "physics.hpp"

namespace oracle {

template <class R> struct EnvOut {
  R obs[MJL_MAXOBS];
  R reward, terminated, truncated;
};

template <class R> R stance_state(const mjlEnvConfig& c, const Data<R>& d) {  // src/envs.py:89-106
  bool r = d.sensordata[c.touch_sensor_right_id] > 0;
  bool l = d.sensordata[c.touch_sensor_left_id] > 0;
  if (r && l) return 0;
  if (r && !l) return 1;
  if (!r && l) return 2;
  return 3;
}

template <class R> void rpy_from_quat(const R* q, R& roll, R& pitch, R& yaw) {  // src/envs.py:357-365
  R w = q[0], x = q[1], y = q[2], z = q[3];
  roll = std::atan2(R(2) * (w * x + y * z), R(1) - R(2) * (x * x + y * y));
  R sinp = R(2) * (w * y - z * x);
  sinp = std::min(std::max(sinp, R(-1)), R(1));
  pitch = std::asin(sinp);
  yaw = std::atan2(R(2) * (w * z + x * y), R(1) - R(2) * (y * y + z * z));
}

// obs assembly (src/envs.py:317-331 with get_body_velocities_local :274-315)
template <class R> void compute_obs(const mjlModelDesc& m, const mjlEnvConfig& c, const Data<R>& d, R flip,
                                    R height, R roll, R pitch, R yaw, const R* q, R tf0, R tf1, R* obs) {
  R w = q[0], x = q[1], y = q[2], z = q[3];
  R r00 = 1 - 2 * (y * y + z * z), r01 = 2 * (x * y - w * z), r02 = 2 * (x * z + w * y);
  R r10 = 2 * (x * y + w * z), r11 = 1 - 2 * (x * x + z * z), r12 = 2 * (y * z - w * x);
  R r20 = 2 * (x * z - w * y), r21 = 2 * (y * z + w * x), r22 = 1 - 2 * (x * x + y * y);
  R raw[MJL_MAXOBS];
  int n = 0;
  raw[n++] = height; raw[n++] = roll; raw[n++] = pitch; raw[n++] = yaw;
  for (int i = 7; i < m.nq; i++) raw[n++] = d.qpos[i];
  for (int h = 0; h < 2; h++) {
    R vx = d.qvel[3 * h], vy = d.qvel[3 * h + 1], vz = d.qvel[3 * h + 2];
    raw[n++] = r00 * vx + r10 * vy + r20 * vz;
    raw[n++] = r01 * vx + r11 * vy + r21 * vz;
    raw[n++] = r02 * vx + r12 * vy + r22 * vz;
  }
  for (int i = 6; i < m.nv; i++) raw[n++] = d.qvel[i];
  raw[n++] = tf0; raw[n++] = tf1;
  for (int i = 0; i < n; i++) obs[i] = flip > R(0.5) ? raw[c.obs_perm[i]] * R(c.obs_sign[i]) : raw[i];
}

template <class R> R xy_dist(R tx, R ty, const R* p) {
  R dx = tx - p[0], dy = ty - p[1];
  return std::sqrt(dx * dx + dy * dy);
}

// single_reset with explicit uniforms u = [joint(nq-7), vel(nv), flip, speed]
template <class R> void env_reset(const mjlModelDesc& m, const mjlEnvConfig& c, Data<R>& d, R* aux,
                                  const R* u, R* obs) {
  make_data(m, d);
  int nj = m.nq - 7;
  for (int i = 0; i < nj; i++) d.qpos[7 + i] += R(c.random_joint_noise) * (u[i] * R(2) - R(1));
  for (int i = 0; i < m.nv; i++) d.qvel[i] = R(c.random_vel_noise) * (u[nj + i] * R(2) - R(1));
  R flip = c.random_flip ? (u[nj + m.nv] < R(0.5) ? R(1) : R(0)) : R(0);
  forward(m, d);
  const R* bp = &d.xpos[3 * c.pelvis_body_id];
  R tx = bp[0] + R(c.target_dist), ty = bp[1], tz = bp[2];
  if (c.initial_velocity_max > 0) {
    R dx = tx - bp[0], dy = ty - bp[1];
    R dxy = std::sqrt(dx * dx + dy * dy);
    R vmag = u[nj + m.nv + 1] * R(c.initial_velocity_max);
    R vx = dxy > R(1e-6) ? vmag * dx / dxy : R(0);
    R vy = dxy > R(1e-6) ? vmag * dy / dxy : R(0);
    d.qvel[0] = vx; d.qvel[1] = vy;
    // single_pipeline_init(qpos, qvel) again: a fresh make_data (qacc_warmstart = 0, src/envs.py:109-113),
    // not the first forward's solution (it matters once the solve is truncated, e.g. CG 4/4)
    std::vector<R> q = d.qpos, v = d.qvel;
    make_data(m, d);
    d.qpos = q; d.qvel = v;
    forward(m, d);
    bp = &d.xpos[3 * c.pelvis_body_id];
  }
  R dxp = tx - bp[0], dyp = ty - bp[1];
  R dist = std::max(xy_dist(tx, ty, bp), xy_dist(tx, ty, &d.xpos[3 * c.head_body_id]));
  R last_pot = -dist / R(m.timestep);
  R stance = stance_state(c, d);
  R a[MJL_AUX_DIM] = {flip, tx, ty, tz, 0, stance, d.time, last_pot, 0};
  for (int i = 0; i < MJL_AUX_DIM; i++) aux[i] = a[i];
  const R* q = &d.xquat[4 * c.pelvis_body_id];
  R roll, pitch, yaw;
  rpy_from_quat(q, roll, pitch, yaw);
  R angle = std::atan2(dyp, dxp) - yaw;
  R soft = dist / (1 + std::abs(dist));
  compute_obs(m, c, d, flip, bp[2], roll, pitch, yaw, q, soft * std::sin(angle), soft * std::cos(angle), obs);
}

template <class R> void env_step(const mjlModelDesc& m, const mjlEnvConfig& c, Data<R>& d, R* aux,
                                 const R* action, EnvOut<R>& out) {
  R flip = aux[0];
  for (int u = 0; u < m.nu; u++) {
    R a = flip > R(0.5) ? action[c.act_perm[u]] * R(c.act_sign[u]) : action[u];
    d.ctrl[u] = std::min(std::max(a, R(-1)), R(1));
  }
  step(m, d);
  const R* hp = &d.xpos[3 * c.head_body_id];
  const R* bp = &d.xpos[3 * c.pelvis_body_id];
  R height = bp[2];
  const R* q = &d.xquat[4 * c.pelvis_body_id];
  R roll, pitch, yaw;
  rpy_from_quat(q, roll, pitch, yaw);
  R tx = aux[1], ty = aux[2], tz = aux[3];
  R dist = std::max(xy_dist(tx, ty, bp), xy_dist(tx, ty, hp));
  R dt = R(m.timestep);
  R progress = (-dist / dt - aux[7]) * R(c.progress_weight);
  R pw = 0, st = 0;
  int nj = m.nv - 6;
  for (int i = 6; i < m.nv; i++) {
    pw += std::abs(d.qfrc_actuator[i] * d.qvel[i]);
    st += d.qfrc_actuator[i] * d.qfrc_actuator[i];
  }
  R energy = R(c.electricity_cost) * (pw / R(nj)) + R(c.stall_torque_cost) * (st / R(nj));
  R posture = ((pitch > R(-0.087)) && (pitch < R(0.174))) ? R(0) : std::abs(pitch);
  posture += ((roll > R(-0.174)) && (roll < R(0.174))) ? R(0) : std::abs(roll);
  posture *= R(c.posture_penalty_weight);
  R tall = R(c.tall_bonus_weight) * (height > R(c.tall_height_threshold) ? R(1) : R(-1));
  R old_st = aux[5], st_time = aux[6];
  R new_st = stance_state(c, d);
  bool changed = new_st != old_st;
  R dur = d.time - st_time;
  R stance_rew = (changed && dur > R(0.1)) ? R(c.stance_time_reward_weight) * dur / dt : R(0);
  R st_upd = changed ? new_st : old_st;
  R st_time_upd = changed ? d.time : st_time;
  bool close = dist < R(c.target_threshold);
  R close_count = close ? aux[4] + 1 : R(0);
  R bonus = close ? R(2) : R(0);
  bool adv = close_count >= R(c.stop_frames);
  if (adv) { tx = bp[0] + R(c.target_dist); ty = bp[1]; tz = bp[2]; close_count = 0; }
  R dxp = tx - bp[0], dyp = ty - bp[1];
  R dist2 = std::max(xy_dist(tx, ty, bp), xy_dist(tx, ty, hp));
  R angle = std::atan2(dyp, dxp) - yaw;
  R soft = dist2 / (1 + std::abs(dist2));
  R reward = progress + bonus + stance_rew - energy + tall - posture;
  R ep = aux[8] + 1;
  bool fallen = height < R(c.terminate_height);
  out.terminated = fallen ? R(1) : R(0);
  out.truncated = (c.max_episode_steps > 0 && ep >= R(c.max_episode_steps)) ? R(1) : R(0);
  if (fallen) reward += R(c.terminate_reward);
  out.reward = reward;
  R a[MJL_AUX_DIM] = {flip, tx, ty, tz, close_count, st_upd, st_time_upd, -dist2 / dt, ep};
  for (int i = 0; i < MJL_AUX_DIM; i++) aux[i] = a[i];
  compute_obs(m, c, d, flip, height, roll, pitch, yaw, q, soft * std::sin(angle), soft * std::cos(angle), out.obs);
}

}  // namespace oracle
