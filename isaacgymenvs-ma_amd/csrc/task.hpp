// task.hpp — fused task layer on gfx950: the reference's @torch.jit.script
// observation/reward functions, reset_idx and the VecTask.step tail, one lane
// per env.  fp32 with FMA contraction disabled so the arithmetic follows the
// reference's per-op rounding (potentials ~ -6e4 are differenced for the
// progress reward, tasks/ant.py:357); transcendentals come from the device
// libm (<= a few ulp from the reference's CPU/ATen implementations).
//
//   quat_mul            utils/torch_jit_utils.py:41-62
//   quat_rotate[_inv]   utils/torch_jit_utils.py:80-103
//   get_euler_xyz       utils/torch_jit_utils.py:175-195
//   compute_heading_and_up / compute_rot   utils/torch_jit_utils.py:247-276
//   compute_ant_observations / _reward     tasks/ant.py:374-408 / :325-371
//   compute_humanoid_observations / _reward tasks/humanoid.py:378-413 / :323-375
//   cartpole obs / reward                 tasks/cartpole.py:131-142 / :180-196
//   reset_idx                             tasks/ant.py:252-279, humanoid.py:253-279, cartpole.py:144-157
#pragma once
#include "../../include/migym.h"
#include "device_math.hpp"

namespace mg {

#pragma clang fp contract(off)

__device__ __forceinline__ void t_quat_mul(const float* a, const float* b, float* o) {
  float x1 = a[0], y1 = a[1], z1 = a[2], w1 = a[3];
  float x2 = b[0], y2 = b[1], z2 = b[2], w2 = b[3];
  float ww = (z1 + x1) * (x2 + y2);
  float yy = (w1 - y1) * (w2 + z2);
  float zz = (w1 + y1) * (w2 - z2);
  float xx = ww + yy + zz;
  float qq = 0.5f * (xx + (z1 - x1) * (x2 - y2));
  o[3] = qq - ww + (z1 - y1) * (y2 - z2);
  o[0] = qq - xx + (x1 + w1) * (x2 + w2);
  o[1] = qq - yy + (w1 - x1) * (y2 + z2);
  o[2] = qq - zz + (z1 + y1) * (w2 - x2);
}
__device__ __forceinline__ void t_quat_rotate(const float* q, const float* v, float* o, bool inverse) {
  float qw = q[3];
  float s = 2.0f * (qw * qw) - 1.0f;
  float c0 = q[1] * v[2] - q[2] * v[1], c1 = q[2] * v[0] - q[0] * v[2], c2 = q[0] * v[1] - q[1] * v[0];
  float c[3] = {c0, c1, c2};
  float d = q[0] * v[0] + q[1] * v[1] + q[2] * v[2];
#pragma unroll
  for (int i = 0; i < 3; i++) {
    float a = v[i] * s;
    float b = c[i] * qw * 2.0f;
    float cc = q[i] * d * 2.0f;
    o[i] = (inverse ? a - b : a + b) + cc;
  }
}
__device__ __forceinline__ float t_mod2pi(float a) {
  const float b = 6.28318530717958647692f;
  float r = fmodf(a, b);
  if (r != 0.0f && (r < 0.0f) != (b < 0.0f)) r += b;
  return r;
}
__device__ __forceinline__ float t_normalize_angle(float x) { return atan2f(sinf(x), cosf(x)); }
__device__ __forceinline__ float t_unscale(float x, float lo, float hi) { return (2.0f * x - hi - lo) / (hi - lo); }

struct LocoFeat {
  float up_proj, heading_proj, up_vec[3], heading_vec[3], vel_loc[3], angvel_loc[3], roll, yaw, angle_to_target,
      potential;
};

__device__ __forceinline__ void loco_features(const mg_task_params* tp, const float* root, const float* off,
                                              LocoFeat& f) {
  const float* pos = root;
  const float tg0 = tp->target[0] + off[0], tg1 = tp->target[1] + off[1], tg2 = tp->target[2] + off[2];
  float tt0 = tg0 - pos[0], tt1 = tg1 - pos[1], tt2 = 0.0f;
  float nrm = sqrtf(tt0 * tt0 + tt1 * tt1 + tt2 * tt2);
  f.potential = -nrm / tp->dt;
  float nc = nrm < 1e-9f ? 1e-9f : nrm;
  float dirs[3] = {tt0 / nc, tt1 / nc, tt2 / nc};
  float inv[4] = {-tp->start_rot[0], -tp->start_rot[1], -tp->start_rot[2], tp->start_rot[3]};
  float tq[4];
  t_quat_mul(root + 3, inv, tq);
  const float b0[3] = {1.0f, 0.0f, 0.0f}, b1[3] = {0.0f, 0.0f, 1.0f};
  t_quat_rotate(tq, b1, f.up_vec, false);
  t_quat_rotate(tq, b0, f.heading_vec, false);
  f.up_proj = f.up_vec[2];
  f.heading_proj = f.heading_vec[0] * dirs[0] + f.heading_vec[1] * dirs[1] + f.heading_vec[2] * dirs[2];
  t_quat_rotate(tq, root + 7, f.vel_loc, true);
  t_quat_rotate(tq, root + 10, f.angvel_loc, true);
  float qx = tq[0], qy = tq[1], qz = tq[2], qw = tq[3];
  float sinr = 2.0f * (qw * qx + qy * qz);
  float cosr = qw * qw - qx * qx - qy * qy + qz * qz;
  f.roll = t_mod2pi(atan2f(sinr, cosr));
  float siny = 2.0f * (qw * qz + qx * qy);
  float cosy = qw * qw + qx * qx - qy * qy - qz * qz;
  f.yaw = t_mod2pi(atan2f(siny, cosy));
  float wta = atan2f(tg2 - pos[2], tg0 - pos[0]);
  f.angle_to_target = wta - f.yaw;
}

__device__ __forceinline__ int t_sensors(const mg_task_params* tp) {
  return tp->task_id == MG_TASK_ANT ? 4 : (tp->task_id == MG_TASK_HUMANOID ? 2 : 0);
}
__device__ __forceinline__ int t_dofs(const mg_task_params* tp) {
  return tp->task_id == MG_TASK_CARTPOLE ? 2 : tp->num_actions;
}

// obs row e (writes potentials/prev_potentials/up/heading like compute_*_observations)
__device__ void obs_env(const mg_task_params* tp, const float* off, const float* root, const float* dof,
                        const float* dof_force, const float* sen, const float* act, float* pot, float* prev_pot,
                        float* up, float* heading, float* o) {
  const int nd = t_dofs(tp), na = tp->num_actions;
  if (tp->task_id == MG_TASK_CARTPOLE) {
    o[0] = dof[0]; o[1] = dof[1]; o[2] = dof[2]; o[3] = dof[3];
    return;
  }
  LocoFeat f;
  loco_features(tp, root, off, f);
  *prev_pot = *pot;
  *pot = f.potential;
  for (int i = 0; i < 3; i++) { up[i] = f.up_vec[i]; heading[i] = f.heading_vec[i]; }
  int k = 0;
  o[k++] = root[2];
  for (int i = 0; i < 3; i++) o[k++] = f.vel_loc[i];
  if (tp->task_id == MG_TASK_ANT) {
    for (int i = 0; i < 3; i++) o[k++] = f.angvel_loc[i];
    o[k++] = f.yaw;
    o[k++] = f.roll;
    o[k++] = f.angle_to_target;
  } else {
    for (int i = 0; i < 3; i++) o[k++] = f.angvel_loc[i] * tp->angular_velocity_scale;
    o[k++] = t_normalize_angle(f.yaw);
    o[k++] = t_normalize_angle(f.roll);
    o[k++] = t_normalize_angle(f.angle_to_target);
  }
  o[k++] = f.up_proj;
  o[k++] = f.heading_proj;
  for (int i = 0; i < nd; i++) o[k++] = t_unscale(dof[2 * i], tp->dof_lower[i], tp->dof_upper[i]);
  for (int i = 0; i < nd; i++) o[k++] = dof[2 * i + 1] * tp->dof_vel_scale;
  if (tp->task_id == MG_TASK_HUMANOID)
    for (int i = 0; i < nd; i++) o[k++] = dof_force[i] * tp->contact_force_scale;
  const int ns = t_sensors(tp);
  for (int i = 0; i < 6 * ns; i++) o[k++] = sen[i] * tp->contact_force_scale;
  for (int i = 0; i < na; i++) o[k++] = act[i];
}

__device__ void reward_env(const mg_task_params* tp, const float* o, const float* a, float pot, float prev_pot,
                           int64_t progress, int64_t* reset, float* rew) {
  const int na = tp->num_actions;
  const float max_ep_m1 = (float)tp->max_episode_length - 1.0f;
  if (tp->task_id == MG_TASK_CARTPOLE) {
    float cart_pos = o[0], cart_vel = o[1], pole_angle = o[2], pole_vel = o[3];
    float r = 1.0f - pole_angle * pole_angle - 0.01f * fabsf(cart_vel) - 0.005f * fabsf(pole_vel);
    const float half_pi = 1.57079632679489661923f;
    int64_t rs = *reset;
    if (fabsf(cart_pos) > tp->reset_dist) { r = -2.0f; rs = 1; }
    if (fabsf(pole_angle) > half_pi) { r = -2.0f; rs = 1; }
    if ((float)progress >= max_ep_m1) rs = 1;
    *rew = r;
    *reset = rs;
    return;
  }
  float heading = o[11] > 0.8f ? tp->heading_weight : tp->heading_weight * o[11] / 0.8f;
  float up = o[10] > 0.93f ? 0.0f + tp->up_weight : 0.0f;
  float ac = 0.0f, el = 0.0f, lim = 0.0f;
  const int nd = na;
  for (int i = 0; i < na; i++) ac += a[i] * a[i];
  if (tp->task_id == MG_TASK_ANT) {
    for (int i = 0; i < na; i++) el += fabsf(a[i] * o[12 + nd + i]);
    int cnt = 0;
    for (int i = 0; i < nd; i++) cnt += o[12 + i] > 0.99f;
    lim = (float)cnt * tp->joints_at_limit_cost_scale;
  } else {
    for (int i = 0; i < nd; i++) {
      float ratio = tp->motor_effort[i] / tp->max_motor_effort;
      float ab = fabsf(o[12 + i]);
      float scaled = tp->joints_at_limit_cost_scale * (ab - 0.98f) / 0.02f;
      lim += (ab > 0.98f ? 1.0f : 0.0f) * scaled * ratio;
      el += fabsf(a[i] * o[12 + nd + i]) * ratio;
    }
  }
  float alive = tp->task_id == MG_TASK_ANT ? 0.5f : 2.0f;
  float progress_reward = pot - prev_pot;
  float total = progress_reward + alive + up + heading - tp->actions_cost_scale * ac - tp->energy_cost_scale * el - lim;
  int64_t rs = *reset;
  if (o[0] < tp->termination_height) { total = tp->death_cost; rs = 1; }
  if ((float)progress >= max_ep_m1) rs = 1;
  *rew = total;
  *reset = rs;
}

// reset_idx for DOF i of one env (ant.py:257-266; cartpole.py:146-151).  noise: row of 2*nD U(0,1)
// (or NULL: device counter RNG)
__device__ __forceinline__ void reset_dof(const mg_task_params* tp, int i, int nd, const float* noise, uint64_t seed,
                                          uint64_t env_gid, uint64_t counter, float* dof) {
  float up = noise ? noise[i] : uniform01(seed, env_gid, counter, (uint32_t)i);
  float uv = noise ? noise[nd + i] : uniform01(seed, env_gid, counter, (uint32_t)(nd + i));
  if (tp->task_id == MG_TASK_CARTPOLE) {
    dof[2 * i] = 0.2f * (up - 0.5f);
    dof[2 * i + 1] = 0.5f * (uv - 0.5f);
  } else {
    float pos = 0.4f * up + -0.2f;
    float vel = 0.2f * uv + -0.1f;
    float q = tp->initial_dof_pos[i] + pos;
    q = q < tp->dof_upper[i] ? q : tp->dof_upper[i];
    q = q > tp->dof_lower[i] ? q : tp->dof_lower[i];
    dof[2 * i] = q;
    dof[2 * i + 1] = vel;
  }
}
// root / potentials part of reset_idx (ant.py:268-279)
__device__ __forceinline__ void reset_root(const mg_task_params* tp, const float* off, float* root, float* pot,
                                           float* prev_pot) {
  if (tp->task_id == MG_TASK_CARTPOLE) return;
  for (int k = 0; k < 3; k++) root[k] = tp->start_pos[k] + off[k];
  for (int k = 0; k < 4; k++) root[3 + k] = tp->start_rot[k];
  for (int k = 7; k < 13; k++) root[k] = 0.0f;
  float t0 = (tp->target[0] + off[0]) - root[0], t1 = (tp->target[1] + off[1]) - root[1], t2 = 0.0f;
  float nrm = sqrtf(t0 * t0 + t1 * t1 + t2 * t2);
  *prev_pot = -nrm / tp->dt;
  *pot = *prev_pot;
}
__device__ void reset_env(const mg_task_params* tp, const float* off, const float* noise, uint64_t seed,
                          uint64_t env_gid, uint64_t counter, float* root, float* dof, float* pot, float* prev_pot) {
  const int nd = t_dofs(tp);
  for (int i = 0; i < nd; i++) reset_dof(tp, i, nd, noise, seed, env_gid, counter, dof);
  reset_root(tp, off, root, pot, prev_pot);
}

// the first 12 observation values of compute_{ant,humanoid}_observations (ant.py:401-406,
// humanoid.py:401-413) + the potentials / basis vectors
__device__ __forceinline__ void obs_head(const mg_task_params* tp, const float* off, const float* root, float* pot,
                                         float* prev_pot, float* up, float* heading, float* o) {
  LocoFeat f;
  loco_features(tp, root, off, f);
  *prev_pot = *pot;
  *pot = f.potential;
  for (int i = 0; i < 3; i++) { up[i] = f.up_vec[i]; heading[i] = f.heading_vec[i]; }
  int k = 0;
  o[k++] = root[2];
  for (int i = 0; i < 3; i++) o[k++] = f.vel_loc[i];
  if (tp->task_id == MG_TASK_ANT) {
    for (int i = 0; i < 3; i++) o[k++] = f.angvel_loc[i];
    o[k++] = f.yaw;
    o[k++] = f.roll;
    o[k++] = f.angle_to_target;
  } else {
    for (int i = 0; i < 3; i++) o[k++] = f.angvel_loc[i] * tp->angular_velocity_scale;
    o[k++] = t_normalize_angle(f.yaw);
    o[k++] = t_normalize_angle(f.roll);
    o[k++] = t_normalize_angle(f.angle_to_target);
  }
  o[k++] = f.up_proj;
  o[k++] = f.heading_proj;
}

// obs_head on a team's first four lanes instead of its leader alone: the same operations on the same operands
// (FMA contraction is off here, so every value is bit-identical to obs_head's), with the per-env serial chain of
// four vector rotations, three atan2 and (Humanoid) three angle normalisations issued once per wave instead of
// one after another.  Lane k of the team: k = 0 rotates e_z (up_vec) and takes the roll, k = 1 rotates e_x
// (heading_vec) and takes the yaw, k = 2 rotates the velocity into the torso frame and takes the walk-target angle
// (then angle_to_target = target angle - yaw), k = 3 rotates the angular velocity; the leader gathers the results
// by shuffles and writes the 12 head entries.  All lanes of the team call it (T >= 4); pot / prev / up / heading
// are valid on the leader.  (compute_heading_and_up / compute_rot, torch_jit_utils.py:247-276; the head of
// compute_{ant,humanoid}_observations, ant.py:398-404, humanoid.py:400-409)
__device__ __forceinline__ void obs_head_team(const mg_task_params* tp, const float* off, const float* root, int tl,
                                              int tb, float* pot, float* prev_pot, float* up, float* heading, float* o) {
  const float* pos = root;
  const float tg0 = tp->target[0] + off[0], tg1 = tp->target[1] + off[1], tg2 = tp->target[2] + off[2];
  float tt0 = tg0 - pos[0], tt1 = tg1 - pos[1], tt2 = 0.0f;
  float nrm = sqrtf(tt0 * tt0 + tt1 * tt1 + tt2 * tt2);
  const float potential = -nrm / tp->dt;
  float inv[4] = {-tp->start_rot[0], -tp->start_rot[1], -tp->start_rot[2], tp->start_rot[3]};
  float tq[4];
  t_quat_mul(root + 3, inv, tq);
  const int k = tl < 4 ? tl : 3;
  // the lane's rotation: e_z, e_x (forward), the linear / angular velocity (inverse)
  float vin[3];
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const float e = (k == 0 && i == 2) || (k == 1 && i == 0) ? 1.0f : 0.0f;
    vin[i] = k < 2 ? e : root[(k == 2 ? 7 : 10) + i];
  }
  float r3[3];
  t_quat_rotate(tq, vin, r3, k >= 2);
  // the lane's angle: roll, yaw (get_euler_xyz, floor-mod 2 pi), the walk-target angle atan2(dz, dx)
  const float qx = tq[0], qy = tq[1], qz = tq[2], qw = tq[3];
  const float sinr = 2.0f * (qw * qx + qy * qz);
  const float cosr = qw * qw - qx * qx - qy * qy + qz * qz;
  const float siny = 2.0f * (qw * qz + qx * qy);
  const float cosy = qw * qw + qx * qx - qy * qy - qz * qz;
  const float ay = k == 0 ? sinr : (k == 1 ? siny : tg2 - pos[2]);
  const float ax = k == 0 ? cosr : (k == 1 ? cosy : tg0 - pos[0]);
  float ang = atan2f(ay, ax);
  if (k < 2) ang = t_mod2pi(ang);
  const float yaw = __shfl(ang, tb + 1);
  if (k == 2) ang = ang - yaw;  // angle_to_target
  const bool hum = tp->task_id != MG_TASK_ANT;
  if (hum) ang = t_normalize_angle(ang);
  const float hv0 = __shfl(r3[0], tb + 1), hv1 = __shfl(r3[1], tb + 1), hv2 = __shfl(r3[2], tb + 1);
  const float vl0 = __shfl(r3[0], tb + 2), vl1 = __shfl(r3[1], tb + 2), vl2 = __shfl(r3[2], tb + 2);
  const float av0 = __shfl(r3[0], tb + 3), av1 = __shfl(r3[1], tb + 3), av2 = __shfl(r3[2], tb + 3);
  const float a1 = __shfl(ang, tb + 1), a2 = __shfl(ang, tb + 2);
  *prev_pot = *pot;
  *pot = potential;
  if (tl != 0) return;
  float nc = nrm < 1e-9f ? 1e-9f : nrm;
  float dirs[3] = {tt0 / nc, tt1 / nc, tt2 / nc};
  for (int i = 0; i < 3; i++) up[i] = r3[i];
  heading[0] = hv0; heading[1] = hv1; heading[2] = hv2;
  o[0] = root[2];
  o[1] = vl0; o[2] = vl1; o[3] = vl2;
  const float avs = hum ? tp->angular_velocity_scale : 1.0f;
  if (hum) {
    o[4] = av0 * avs; o[5] = av1 * avs; o[6] = av2 * avs;
  } else {
    o[4] = av0; o[5] = av1; o[6] = av2;
  }
  o[7] = a1;   // yaw
  o[8] = ang;  // roll (the leader's own angle)
  o[9] = a2;   // angle_to_target
  o[10] = r3[2];
  o[11] = hv0 * dirs[0] + hv1 * dirs[1] + hv2 * dirs[2];
}

// reward given the team sums of the per-action terms (compute_{ant,humanoid}_reward, ant.py:325-371,
// humanoid.py:323-375); ac = sum a^2, el = energy term, lim = joints-at-limit term
__device__ __forceinline__ void reward_from_sums(const mg_task_params* tp, const float* o, float ac, float el,
                                                 float lim, float pot, float prev_pot, int64_t progress,
                                                 int64_t* reset, float* rew) {
  const float max_ep_m1 = (float)tp->max_episode_length - 1.0f;
  float heading = o[11] > 0.8f ? tp->heading_weight : tp->heading_weight * o[11] / 0.8f;
  float up = o[10] > 0.93f ? 0.0f + tp->up_weight : 0.0f;
  float alive = tp->task_id == MG_TASK_ANT ? 0.5f : 2.0f;
  float progress_reward = pot - prev_pot;
  float total = progress_reward + alive + up + heading - tp->actions_cost_scale * ac - tp->energy_cost_scale * el - lim;
  int64_t rs = *reset;
  if (o[0] < tp->termination_height) { total = tp->death_cost; rs = 1; }
  if ((float)progress >= max_ep_m1) rs = 1;
  *rew = total;
  *reset = rs;
}

__device__ __forceinline__ float clampf(float x, float lim) {
  x = x < lim ? x : lim;
  return x > -lim ? x : -lim;
}

#pragma clang fp contract(fast)

}  // namespace mg
