/*
 * oracle_task.c — CPU restatement of the reference's task layer.  TEST
 * INFRASTRUCTURE ONLY (tests/, smoke(), bench.py cpu_baseline).
 *
 * PINNED against the reference's own outputs (tests/golden/jit_*.npz and
 * trace_*.npz).  Arithmetic is fp32 with the reference's operation order
 * (built with -ffp-contract=off) because the reference computes in fp32 and
 * some quantities cancel catastrophically (potentials ~ -6e4, their
 * difference ~1e-2 is the progress reward: tasks/ant.py:357).
 *
 * Restated functions (reference file:line):
 *   quat_mul            utils/torch_jit_utils.py:41-62 (factored 8-multiply form)
 *   normalize           utils/torch_jit_utils.py:65-67
 *   quat_rotate[_inv]   utils/torch_jit_utils.py:80-103
 *   normalize_angle     utils/torch_jit_utils.py:126-128
 *   get_euler_xyz       utils/torch_jit_utils.py:175-195 (Python floor-mod 2pi)
 *   unscale             utils/torch_jit_utils.py:239-240
 *   compute_heading_and_up / compute_rot   utils/torch_jit_utils.py:247-276
 *   compute_ant_observations / _reward     tasks/ant.py:374-408 / :325-371
 *   compute_humanoid_observations / _reward tasks/humanoid.py:378-413 / :323-375
 *   cartpole obs / compute_cartpole_reward tasks/cartpole.py:131-142 / :180-196
 *   reset_idx            tasks/ant.py:252-279, humanoid.py:253-279, cartpole.py:144-157
 *   post_physics_step    tasks/ant.py:287-297 (progress, reset, obs, reward)
 *   VecTask.step tail    tasks/base/vec_task.py:393-410 (timeout, obs clamp)
 */
#include <math.h>
#include <string.h>

#include "oracle.h"

#define PI_F 3.14159265358979323846f

/* ---------------------------------------------------------------- RNG */
static uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
float orc_uniform(uint64_t seed, uint64_t env, uint64_t counter, uint32_t k) {
  uint64_t h = mix64(mix64(mix64(seed ^ (env * 0xD2B74407B1CE6E93ull)) ^ counter) ^ (uint64_t)k);
  return (float)(h >> 40) * (1.0f / 16777216.0f);
}

/* ---------------------------------------------------------------- fp32 helpers */
static void f_quat_mul(const float* a, const float* b, float* o) {
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
static void f_cross(const float* a, const float* b, float* o) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}
static void f_quat_rotate(const float* q, const float* v, float* o, int inverse) {
  float qw = q[3];
  float s = 2.0f * (qw * qw) - 1.0f;
  float c[3];
  f_cross(q, v, c);
  float d = q[0] * v[0] + q[1] * v[1] + q[2] * v[2];
  for (int i = 0; i < 3; i++) {
    float a = v[i] * s;
    float b = c[i] * qw * 2.0f;
    float cc = q[i] * d * 2.0f;
    o[i] = (inverse ? a - b : a + b) + cc;
  }
}
static float f_mod2pi(float a) { /* torch remainder(a, 2*pi) */
  const float b = (float)(2.0 * 3.14159265358979323846);
  float r = fmodf(a, b);
  if (r != 0.0f && (r < 0.0f) != (b < 0.0f)) r += b;
  return r;
}
static void f_euler_xyz(const float* q, float* roll, float* pitch, float* yaw) {
  float qx = q[0], qy = q[1], qz = q[2], qw = q[3];
  float sinr = 2.0f * (qw * qx + qy * qz);
  float cosr = qw * qw - qx * qx - qy * qy + qz * qz;
  *roll = f_mod2pi(atan2f(sinr, cosr));
  float sinp = 2.0f * (qw * qy - qz * qx);
  float p = fabsf(sinp) >= 1.0f ? copysignf(PI_F / 2.0f, sinp) : asinf(sinp);
  *pitch = f_mod2pi(p);
  float siny = 2.0f * (qw * qz + qx * qy);
  float cosy = qw * qw + qx * qx - qy * qy - qz * qz;
  *yaw = f_mod2pi(atan2f(siny, cosy));
}
static float f_normalize_angle(float x) { return atan2f(sinf(x), cosf(x)); }
static float f_unscale(float x, float lo, float hi) { return (2.0f * x - hi - lo) / (hi - lo); }

/* compute_heading_and_up + compute_rot for one env; returns features */
typedef struct {
  float torso_quat[4], up_proj, heading_proj, up_vec[3], heading_vec[3];
  float vel_loc[3], angvel_loc[3], roll, pitch, yaw, angle_to_target;
  float potential;
} loco_feat;

static void loco_features(const mg_task_params* tp, const float* root, const float* inv_start, const float* off,
                          loco_feat* f) {
  const float* pos = root;
  const float* rot = root + 3;
  const float tg[3] = {tp->target[0] + off[0], tp->target[1] + off[1], tp->target[2] + off[2]};
  float to_target[3] = {tg[0] - pos[0], tg[1] - pos[1], 0.0f};
  float nrm = sqrtf(to_target[0] * to_target[0] + to_target[1] * to_target[1] + to_target[2] * to_target[2]);
  f->potential = -nrm / tp->dt;
  float nc = nrm < 1e-9f ? 1e-9f : nrm;
  float dirs[3] = {to_target[0] / nc, to_target[1] / nc, to_target[2] / nc};
  f_quat_mul(rot, inv_start, f->torso_quat);
  const float b0[3] = {1.0f, 0.0f, 0.0f}, b1[3] = {0.0f, 0.0f, 1.0f};
  f_quat_rotate(f->torso_quat, b1, f->up_vec, 0);
  f_quat_rotate(f->torso_quat, b0, f->heading_vec, 0);
  f->up_proj = f->up_vec[2];
  f->heading_proj = f->heading_vec[0] * dirs[0] + f->heading_vec[1] * dirs[1] + f->heading_vec[2] * dirs[2];
  f_quat_rotate(f->torso_quat, root + 7, f->vel_loc, 1);
  f_quat_rotate(f->torso_quat, root + 10, f->angvel_loc, 1);
  f_euler_xyz(f->torso_quat, &f->roll, &f->pitch, &f->yaw);
  float wta = atan2f(tg[2] - pos[2], tg[0] - pos[0]);
  f->angle_to_target = wta - f->yaw;
}

static void inv_start_rot(const mg_task_params* tp, float* q) {
  q[0] = -tp->start_rot[0]; q[1] = -tp->start_rot[1]; q[2] = -tp->start_rot[2]; q[3] = tp->start_rot[3];
}

static int sensors_per_env(const mg_task_params* tp) {
  return tp->task_id == MG_TASK_ANT ? 4 : (tp->task_id == MG_TASK_HUMANOID ? 2 : 0);
}
static int dofs_of(const mg_task_params* tp) { return tp->task_id == MG_TASK_CARTPOLE ? 2 : tp->num_actions; }

static void obs_one(const mg_task_params* tp, int e, const float* root_states, const float* dof_state,
                    const float* dof_force, const float* sensors, const float* actions, float* potentials,
                    float* prev_potentials, float* up_vec, float* heading_vec, float* obs) {
  int nd = dofs_of(tp), na = tp->num_actions, no = tp->num_obs;
  const float* dof = dof_state + 2 * nd * e;
  float* o = obs + (size_t)no * e;
  if (tp->task_id == MG_TASK_CARTPOLE) {
    o[0] = dof[0]; o[1] = dof[1]; o[2] = dof[2]; o[3] = dof[3];
    return;
  }
  const float* root = root_states + 13 * e;
  const int A = tp->num_agents > 1 ? tp->num_agents : 1;
  const float* off = tp->agent_offset[e % A];
  float inv[4];
  inv_start_rot(tp, inv);
  loco_feat f;
  loco_features(tp, root, inv, off, &f);
  prev_potentials[e] = potentials[e];
  potentials[e] = f.potential;
  for (int i = 0; i < 3; i++) { up_vec[3 * e + i] = f.up_vec[i]; heading_vec[3 * e + i] = f.heading_vec[i]; }
  int ns = sensors_per_env(tp);
  const float* sen = sensors + 6 * ns * e;
  const float* act = actions + (size_t)na * e;
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
    o[k++] = f_normalize_angle(f.yaw);
    o[k++] = f_normalize_angle(f.roll);
    o[k++] = f_normalize_angle(f.angle_to_target);
  }
  o[k++] = f.up_proj;
  o[k++] = f.heading_proj;
  for (int i = 0; i < nd; i++) o[k++] = f_unscale(dof[2 * i], tp->dof_lower[i], tp->dof_upper[i]);
  for (int i = 0; i < nd; i++) o[k++] = dof[2 * i + 1] * tp->dof_vel_scale;
  if (tp->task_id == MG_TASK_HUMANOID)
    for (int i = 0; i < nd; i++) o[k++] = dof_force[(size_t)nd * e + i] * tp->contact_force_scale;
  for (int i = 0; i < 6 * ns; i++) o[k++] = sen[i] * tp->contact_force_scale;
  for (int i = 0; i < na; i++) o[k++] = act[i];
  if (A > 1) {  /* others, cyclic shift after self (franka_reach_MA.py:604-608), relative to self */
    const int ag = e % A, base = e - ag;
    for (int j = 1; j < A; j++) {
      const float* q = root_states + 13 * (base + (ag + j) % A);
      for (int c = 0; c < 3; c++) o[k++] = q[c] - root[c];
    }
  }
}

int orc_compute_observations(const mg_task_params* tp, int32_t n, const float* root_states, const float* dof_state,
                             const float* dof_force, const float* sensors, const float* actions,
                             float* potentials, float* prev_potentials, float* up_vec, float* heading_vec,
                             float* obs) {
  for (int e = 0; e < n; e++)
    obs_one(tp, e, root_states, dof_state, dof_force, sensors, actions, potentials, prev_potentials, up_vec,
            heading_vec, obs);
  return 0;
}

static void reward_one(const mg_task_params* tp, int e, const float* obs, const float* actions,
                       const float* potentials, const float* prev_potentials, const int64_t* progress,
                       int64_t* reset, float* rew) {
  int na = tp->num_actions, no = tp->num_obs;
  const float* o = obs + (size_t)no * e;
  const float* a = actions + (size_t)na * e;
  float max_ep_m1 = (float)tp->max_episode_length - 1.0f;
  if (tp->task_id == MG_TASK_CARTPOLE) {
    float cart_pos = o[0], cart_vel = o[1], pole_angle = o[2], pole_vel = o[3];
    float r = 1.0f - pole_angle * pole_angle - 0.01f * fabsf(cart_vel) - 0.005f * fabsf(pole_vel);
    const float half_pi = (float)(3.14159265358979323846 / 2.0);
    int64_t rs = reset[e];
    if (fabsf(cart_pos) > tp->reset_dist) { r = -2.0f; rs = 1; }
    if (fabsf(pole_angle) > half_pi) { r = -2.0f; rs = 1; }
    if ((float)progress[e] >= max_ep_m1) rs = 1;
    rew[e] = r;
    reset[e] = rs;
    return;
  }
  float heading = o[11] > 0.8f ? tp->heading_weight : tp->heading_weight * o[11] / 0.8f;
  float up = o[10] > 0.93f ? 0.0f + tp->up_weight : 0.0f;
  float ac = 0.0f, el = 0.0f, lim = 0.0f;
  int nd = na;
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
  float progress_reward = potentials[e] - prev_potentials[e];
  float total = progress_reward + alive + up + heading - tp->actions_cost_scale * ac - tp->energy_cost_scale * el - lim;
  int64_t rs = reset[e];
  if (o[0] < tp->termination_height) { total = tp->death_cost; rs = 1; }
  if ((float)progress[e] >= max_ep_m1) rs = 1;
  rew[e] = total;
  reset[e] = rs;
}

int orc_compute_reward(const mg_task_params* tp, int32_t n, const float* obs, const float* actions,
                       const float* potentials, const float* prev_potentials, const int64_t* progress,
                       int64_t* reset, float* rew) {
  for (int e = 0; e < n; e++) reward_one(tp, e, obs, actions, potentials, prev_potentials, progress, reset, rew);
  return 0;
}

/* reset_idx for one env (noise = raw U(0,1) draws: [pos(nD), vel(nD)]) */
static void reset_one(const mg_task_params* tp, int e, const mg_state_views* v, const mg_task_buffers* tb) {
  int nd = dofs_of(tp);
  float u[128];
  for (int k = 0; k < 2 * nd; k++)
    u[k] = tb->noise ? tb->noise[(size_t)2 * nd * e + k]
                     : orc_uniform(tb->seed, (uint64_t)(tb->env_offset * (tp->num_agents > 1 ? tp->num_agents : 1) + e),
                                   tb->step_counter, (uint32_t)k);
  float* dof = v->dof_state + 2 * nd * e;
  if (tp->task_id == MG_TASK_CARTPOLE) {
    for (int i = 0; i < nd; i++) {
      dof[2 * i] = 0.2f * (u[i] - 0.5f);
      dof[2 * i + 1] = 0.5f * (u[nd + i] - 0.5f);
    }
  } else {
    for (int i = 0; i < nd; i++) {
      float pos = 0.4f * u[i] + -0.2f;
      float vel = 0.2f * u[nd + i] + -0.1f;
      float q = tp->initial_dof_pos[i] + pos;
      q = q < tp->dof_upper[i] ? q : tp->dof_upper[i];
      q = q > tp->dof_lower[i] ? q : tp->dof_lower[i];
      dof[2 * i] = q;
      dof[2 * i + 1] = vel;
    }
    const int A = tp->num_agents > 1 ? tp->num_agents : 1;
    const float* off = tp->agent_offset[e % A];
    float* root = v->root_states + 13 * e;
    for (int k = 0; k < 3; k++) root[k] = tp->start_pos[k] + off[k];
    for (int k = 0; k < 4; k++) root[3 + k] = tp->start_rot[k];
    for (int k = 7; k < 13; k++) root[k] = 0.0f;
    float tt[3] = {(tp->target[0] + off[0]) - root[0], (tp->target[1] + off[1]) - root[1], 0.0f};
    float nrm = sqrtf(tt[0] * tt[0] + tt[1] * tt[1] + tt[2] * tt[2]);
    tb->prev_potentials[e] = -nrm / tp->dt;
    tb->potentials[e] = tb->prev_potentials[e];
  }
  tb->progress[e] = 0;
  tb->reset[e] = 0;
}

int orc_post_physics(const mg_task_params* tp, const mg_state_views* v, const mg_task_buffers* tb, int32_t n) {
  int na = tp->num_actions, no = tp->num_obs;
  const int A = tp->num_agents > 1 ? tp->num_agents : 1;
  float* act = tb->actions_out;
  for (int base = 0; base < n; base += A) {
    /* env resets only when all its agents are done (AND filter, franka_reach_MA.py:875-885) */
    int all_done = 1;
    for (int k = 0; k < A; k++) all_done &= tb->reset[base + k] != 0;
    for (int e = base; e < base + A; e++) {
      for (int i = 0; i < na; i++) {
        float a = tb->actions[(size_t)na * e + i];
        a = a < tp->clip_actions ? a : tp->clip_actions;
        a = a > -tp->clip_actions ? a : -tp->clip_actions;
        act[(size_t)na * e + i] = a;
      }
      tb->progress[e] += 1;
      if (all_done) reset_one(tp, e, v, tb);
    }
    for (int e = base; e < base + A; e++) {
      obs_one(tp, e, v->root_states, v->dof_state, v->dof_force, v->sensors, act, tb->potentials,
              tb->prev_potentials, tb->up_vec, tb->heading_vec, tb->obs);
      reward_one(tp, e, tb->obs, act, tb->potentials, tb->prev_potentials, tb->progress, tb->reset, tb->rew);
      float max_ep_m1 = (float)tp->max_episode_length - 1.0f;
      tb->timeout[e] = (uint8_t)(((float)tb->progress[e] >= max_ep_m1) && (tb->reset[e] != 0));
      if (tb->obs_clamped)
        for (int i = 0; i < no; i++) {
          float x = tb->obs[(size_t)no * e + i];
          x = x < tp->clip_obs ? x : tp->clip_obs;
          x = x > -tp->clip_obs ? x : -tp->clip_obs;
          tb->obs_clamped[(size_t)no * e + i] = x;
        }
    }
  }
  return 0;
}

/* reset_idx(ids) applied now (ant.py:252-279, humanoid.py:253-279, cartpole.py:144-157), the counterpart of
   mg_reset_idx: ids < 0 or >= n are skipped (the AND-filtered multi-agent rows); the counter RNG runs on its
   manual-reset stream (step_counter | 2^62), injected noise rows are indexed by actor. */
int orc_reset_idx(const mg_task_params* tp, const mg_state_views* v, const mg_task_buffers* tb, const int32_t* ids,
                  int32_t n_ids, int32_t n) {
  if (tp->task_id == MG_TASK_SHADOW_HAND) return -1;
  mg_task_buffers t = *tb;
  t.step_counter = tb->step_counter | (1ull << 62);
  for (int k = 0; k < n_ids; k++)
    if (ids[k] >= 0 && ids[k] < n) reset_one(tp, ids[k], v, &t);
  return 0;
}

int orc_env_step(const mg_model* m, const mg_sim_params* p, const mg_task_params* tp, const mg_state_views* v,
                 const mg_task_buffers* tb, int32_t n, int32_t threads) {
  int na = tp->num_actions, nd = m->num_dofs;
  /* pre_physics_step: clamp, effort = a * gear * power_scale (ant.py:281-285; cartpole.py:159-163) */
  float* eff = v->dof_actuation ? (float*)v->dof_actuation : 0;
  if (eff) {
    for (int e = 0; e < n; e++)
      for (int i = 0; i < nd; i++) {
        float a = 0.0f;
        int ai = tp->task_id == MG_TASK_CARTPOLE ? (i == 0 ? 0 : -1) : i;
        if (ai >= 0) {
          a = tb->actions[(size_t)na * e + ai];
          a = a < tp->clip_actions ? a : tp->clip_actions;
          a = a > -tp->clip_actions ? a : -tp->clip_actions;
        }
        eff[(size_t)nd * e + i] = tp->task_id == MG_TASK_CARTPOLE ? a * tp->power_scale
                                                                    : a * tp->motor_effort[i] * tp->power_scale;
      }
  }
  /* gym.simulate x controlFrequencyInv (vec_task.py:381-384) */
  for (int k = 0; k < (tp->control_freq_inv > 1 ? tp->control_freq_inv : 1); k++)
    orc_simulate(m, p, n, v->root_states, v->dof_state, eff, v->sensors, v->dof_force, threads);
  return orc_post_physics(tp, v, tb, n);
}
