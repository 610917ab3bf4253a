// hand_task.hpp — the ShadowHand task layer on gfx950:
// the reference's @torch.jit.script reward, randomize_rotation and the tensor code of
// pre_physics_step / reset_idx / compute_full_state, per env.  fp32 with FMA contraction off,
// in the reference's operation order (same rules as task.hpp).
//
//   quat_from_angle_axis / quat_conjugate   utils/torch_jit_utils.py:107-123
//   scale / tensor_clamp / unscale          utils/torch_jit_utils.py:229-240
//   randomize_rotation                      tasks/shadow_hand.py:803-806
//   randomize_rotation_pen                  tasks/shadow_hand.py:810-813
//   compute_hand_reward                     tasks/shadow_hand.py:746-800
//   compute_full_state                      tasks/shadow_hand.py:528-584
//   reset_target_pose / reset_idx           tasks/shadow_hand.py:586-668
//   pre_physics_step                        tasks/shadow_hand.py:670-698
#pragma once
#include "../../include/migym.h"
#include "device_math.hpp"
#include "task.hpp"

namespace mg {

#pragma clang fp contract(off)

// injected noise row: [goal-only 4 | reset_idx 53 | reset_target_pose 4 | force-probability redraw 1 |
// force selection 1 | force direction 3 (N(0,1))]  (shadow_hand.py:587, 610, 642-643, 704-706)
constexpr int HAND_NOISE = 66;
constexpr int HN_FORCE_PROB = 61, HN_FORCE_SEL = 62, HN_FORCE_DIR = 63;

// observation layouts of observationType (shadow_hand.py:108-113, 473-584): segment lists
enum HandSeg {
  HS_DOF_POS, HS_DOF_VEL, HS_DOF_FORCE, HS_OBJ_POSE, HS_OBJ_POS, HS_OBJ_LINVEL, HS_OBJ_ANGVEL, HS_GOAL_POSE,
  HS_QUAT_DIFF, HS_FT_STATE, HS_FT_POS, HS_FT_FORCE, HS_ACTIONS, HS_END
};
// 0 full_state (compute_full_state, 211), 1 full (157), 2 full_no_vel (77), 3 openai (42)
__constant__ const int8_t kHandLayout[4][12] = {
    {HS_DOF_POS, HS_DOF_VEL, HS_DOF_FORCE, HS_OBJ_POSE, HS_OBJ_LINVEL, HS_OBJ_ANGVEL, HS_GOAL_POSE, HS_QUAT_DIFF,
     HS_FT_STATE, HS_FT_FORCE, HS_ACTIONS, HS_END},
    {HS_DOF_POS, HS_DOF_VEL, HS_OBJ_POSE, HS_OBJ_LINVEL, HS_OBJ_ANGVEL, HS_GOAL_POSE, HS_QUAT_DIFF, HS_FT_STATE,
     HS_ACTIONS, HS_END, HS_END, HS_END},
    {HS_DOF_POS, HS_OBJ_POSE, HS_GOAL_POSE, HS_QUAT_DIFF, HS_FT_POS, HS_ACTIONS, HS_END, HS_END, HS_END, HS_END,
     HS_END, HS_END},
    {HS_FT_POS, HS_OBJ_POS, HS_QUAT_DIFF, HS_ACTIONS, HS_END, HS_END, HS_END, HS_END, HS_END, HS_END, HS_END, HS_END}};

__device__ __forceinline__ int h_seg_size(int seg, int nd, int nf, int na) {
  switch (seg) {
    case HS_DOF_POS: case HS_DOF_VEL: case HS_DOF_FORCE: return nd;
    case HS_OBJ_POSE: case HS_GOAL_POSE: return 7;
    case HS_OBJ_POS: case HS_OBJ_LINVEL: case HS_OBJ_ANGVEL: return 3;
    case HS_QUAT_DIFF: return 4;
    case HS_FT_STATE: return 13 * nf;
    case HS_FT_POS: return 3 * nf;
    case HS_FT_FORCE: return 6 * nf;
    case HS_ACTIONS: return na;
    default: return 0;
  }
}
// observation column k -> (segment, index within the segment)
__device__ __forceinline__ int h_locate_in(int layout, const mg_task_params& tp, int nd, int k, int* idx) {
  const int8_t* lay = kHandLayout[layout & 3];
  for (int i = 0; i < 12 && lay[i] != HS_END; i++) {
    const int n = h_seg_size(lay[i], nd, tp.num_fingertips, tp.num_actions);
    if (k < n) { *idx = k; return lay[i]; }
    k -= n;
  }
  *idx = 0;
  return HS_END;
}
__device__ __forceinline__ int h_locate(const mg_task_params& tp, int nd, int k, int* idx) {
  return h_locate_in(tp.obs_type, tp, nd, k, idx);
}
// host copy of the layouts: fills obs_map / state_map (column -> segment << 8 | index) once per launch,
// so the kernels look a column up instead of walking the segment list per column
static const int8_t kHandLayoutHost[4][12] = {
    {HS_DOF_POS, HS_DOF_VEL, HS_DOF_FORCE, HS_OBJ_POSE, HS_OBJ_LINVEL, HS_OBJ_ANGVEL, HS_GOAL_POSE, HS_QUAT_DIFF,
     HS_FT_STATE, HS_FT_FORCE, HS_ACTIONS, HS_END},
    {HS_DOF_POS, HS_DOF_VEL, HS_OBJ_POSE, HS_OBJ_LINVEL, HS_OBJ_ANGVEL, HS_GOAL_POSE, HS_QUAT_DIFF, HS_FT_STATE,
     HS_ACTIONS, HS_END, HS_END, HS_END},
    {HS_DOF_POS, HS_OBJ_POSE, HS_GOAL_POSE, HS_QUAT_DIFF, HS_FT_POS, HS_ACTIONS, HS_END, HS_END, HS_END, HS_END,
     HS_END, HS_END},
    {HS_FT_POS, HS_OBJ_POS, HS_QUAT_DIFF, HS_ACTIONS, HS_END, HS_END, HS_END, HS_END, HS_END, HS_END, HS_END, HS_END}};
inline int h_seg_size_host(int seg, int nd, int nf, int na) {
  switch (seg) {
    case HS_DOF_POS: case HS_DOF_VEL: case HS_DOF_FORCE: return nd;
    case HS_OBJ_POSE: case HS_GOAL_POSE: return 7;
    case HS_OBJ_POS: case HS_OBJ_LINVEL: case HS_OBJ_ANGVEL: return 3;
    case HS_QUAT_DIFF: return 4;
    case HS_FT_STATE: return 13 * nf;
    case HS_FT_POS: return 3 * nf;
    case HS_FT_FORCE: return 6 * nf;
    case HS_ACTIONS: return na;
    default: return 0;
  }
}
inline void h_fill_map(uint16_t* map, int layout, int nd, int nf, int na) {
  int k = 0;
  for (int i = 0; i < 12 && kHandLayoutHost[layout & 3][i] != HS_END && k < 256; i++) {
    const int seg = kHandLayoutHost[layout & 3][i], n = h_seg_size_host(seg, nd, nf, na);
    for (int j = 0; j < n && k < 256; j++) map[k++] = (uint16_t)((seg << 8) | j);
  }
  for (; k < 256; k++) map[k] = (uint16_t)(HS_END << 8);
}
inline void h_fill_maps(mg_task_params* tp) {
  h_fill_map(tp->obs_map, tp->obs_type, tp->num_dofs, tp->num_fingertips, tp->num_actions);
  h_fill_map(tp->state_map, 0, tp->num_dofs, tp->num_fingertips, tp->num_actions);
}

// fingertip body / component of an HS_FT_STATE or HS_FT_POS index
__device__ __forceinline__ void h_ft_ref(const mg_task_params& tp, int seg, int idx, int* body, int* comp) {
  const int w = seg == HS_FT_STATE ? 13 : 3;
  *body = tp.fingertip_body[idx / w];
  *comp = idx % w;
}
// value of a non-fingertip segment entry
__device__ __forceinline__ float h_obs_value(const mg_task_params& tp, int seg, int i, const float* dof,
                                             const float* dforce, const float* orow, const float* gs,
                                             const float* qdiff, const float* sens, const float* act) {
  switch (seg) {
    case HS_DOF_POS: return (2.0f * dof[2 * i] - tp.dof_upper[i] - tp.dof_lower[i]) / (tp.dof_upper[i] - tp.dof_lower[i]);
    case HS_DOF_VEL: return tp.vel_obs_scale * dof[2 * i + 1];
    case HS_DOF_FORCE: return tp.force_torque_obs_scale * dforce[i];
    case HS_OBJ_POSE: case HS_OBJ_POS: return orow[i];
    case HS_OBJ_LINVEL: return orow[7 + i];
    case HS_OBJ_ANGVEL: return tp.vel_obs_scale * orow[10 + i];
    case HS_GOAL_POSE: return gs[i];
    case HS_QUAT_DIFF: return qdiff[i];
    case HS_FT_FORCE: return tp.force_torque_obs_scale * sens[i];
    case HS_ACTIONS: return act[i];
    default: return 0.0f;
  }
}

__device__ __forceinline__ void h_quat_from_angle_axis(float angle, int k, float* q) {
  const float theta = angle / 2.0f;
  const float sn = sinf(theta), c = cosf(theta);
  float v[4] = {0.0f, 0.0f, 0.0f, c};
  v[k] = 1.0f * sn;
  float n = sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3]);
  n = n < 1e-9f ? 1e-9f : n;
  for (int i = 0; i < 4; i++) q[i] = v[i] / n;
}

__device__ __forceinline__ void h_randomize_rotation(float r0, float r1, float* q) {
  const float pi = 3.14159265358979323846f;
  float qa[4], qb[4];
  h_quat_from_angle_axis(r0 * pi, 0, qa);
  h_quat_from_angle_axis(r1 * pi, 1, qb);
  t_quat_mul(qa, qb, q);
}

// randomize_rotation_pen(rand0, rand1, max_angle = tensor(0.3), x, y, z) (shadow_hand.py:810-813); rand1 is
// unused, as in the reference
__device__ __forceinline__ void h_randomize_rotation_pen(float r0, float* q) {
  const float pi = 3.14159265358979323846f;
  float qa[4], qb[4];
  h_quat_from_angle_axis((float)(0.5 * 3.14159265358979323846) + r0 * 0.3f, 0, qa);
  h_quat_from_angle_axis(r0 * pi, 2, qb);
  t_quat_mul(qa, qb, q);
}

// the object's reset orientation (shadow_hand.py:625-629): pen (ignore_z_rot) or generic
__device__ __forceinline__ void h_object_reset_rotation(const mg_task_params& tp, float r0, float r1, float* q) {
  if (tp.ignore_z_rot) h_randomize_rotation_pen(r0, q);
  else h_randomize_rotation(r0, r1, q);
}

__device__ __forceinline__ float h_rand_pm1(float u) { return 2.0f * u + -1.0f; }

// uniform k of env `gid` for this control step: injected noise row or the counter-based RNG
__device__ __forceinline__ float h_uniform(const mg_task_buffers& tb, int e, uint64_t gid, int k) {
  return tb.noise ? tb.noise[(size_t)HAND_NOISE * e + k] : uniform01(tb.seed, gid, tb.step_counter, (uint32_t)k);
}

// N(0,1) draw k of env `gid`: injected noise column, or Box-Muller on two counter-based uniforms
__device__ __forceinline__ float h_normal(const mg_task_buffers& tb, int e, uint64_t gid, int k) {
  if (tb.noise) return tb.noise[(size_t)HAND_NOISE * e + k];
  const float u1 = uniform01(tb.seed, gid, tb.step_counter, (uint32_t)(128 + 2 * k));
  const float u2 = uniform01(tb.seed, gid, tb.step_counter, (uint32_t)(129 + 2 * k));
  return sqrtf(-2.0f * logf(1.0f - u1)) * cosf(6.28318530717958647f * u2);
}

// random object force of one env for this step (shadow_hand.py:641-643 in reset_idx, 700-706 in
// pre_physics_step): a reset zeroes the force and redraws the env's probability
// exp((log lo - log hi) u + log hi); then, with forceScale > 0, the force decays by
// forceDecay^(dt / forceDecayInterval) (tp.force_decay_step, evaluated on the host with torch.pow) and
// with probability `prob` is replaced by N(0,1)^3 * object mass * forceScale.  f: in/out (3).
__device__ __forceinline__ void h_object_force(const mg_task_params& tp, const mg_task_buffers& tb, int e,
                                               uint64_t gid, bool env_reset, float* f) {
  float prob = tb.random_force_prob ? tb.random_force_prob[e] : 0.0f;
  if (env_reset) {
    f[0] = f[1] = f[2] = 0.0f;
    const float lhi = logf(tp.force_prob_hi);
    prob = expf((logf(tp.force_prob_lo) - lhi) * h_uniform(tb, e, gid, HN_FORCE_PROB) + lhi);
    if (tb.random_force_prob) tb.random_force_prob[e] = prob;
  }
  if (tp.force_scale > 0.0f) {
    for (int k = 0; k < 3; k++) f[k] = f[k] * tp.force_decay_step;
    if (h_uniform(tb, e, gid, HN_FORCE_SEL) < prob)
      for (int k = 0; k < 3; k++) f[k] = h_normal(tb, e, gid, HN_FORCE_DIR + k) * tp.object_rb_mass * tp.force_scale;
  }
}

// reset_target_pose: goal_states (13) and the goal actor's root row (13)
__device__ __forceinline__ void h_reset_goal(const mg_task_params& tp, float g0, float g1, float* gs, float* groot) {
  float q[4];
  h_randomize_rotation(g0, g1, q);
  gs[0] = tp.object_start[0];
  gs[1] = tp.object_start[1];
  gs[2] = tp.object_start[2] + tp.goal_dz;
  for (int k = 0; k < 4; k++) gs[3 + k] = q[k];
  for (int k = 0; k < 3; k++) groot[k] = gs[k] + tp.goal_displacement[k];
  for (int k = 0; k < 4; k++) groot[3 + k] = q[k];
  for (int k = 7; k < 13; k++) groot[k] = 0.0f;
}

// compute_hand_reward for one env (the global running mean is reduced by the caller)
__device__ __forceinline__ void h_reward(const mg_task_params& tp, const float* opos, const float* orot,
                                         const float* tpos, const float* trot, const float* act, int64_t reset_in,
                                         int64_t goal_in, int64_t* progress, float* successes, float* rew,
                                         int64_t* reset_out, int64_t* goal_out) {
  const float max_episode_length = (float)tp.max_episode_length;
  const float d0 = opos[0] - tpos[0], d1 = opos[1] - tpos[1], d2 = opos[2] - tpos[2];
  const float goal_dist = sqrtf(d0 * d0 + d1 * d1 + d2 * d2);
  float tol = tp.success_tolerance;
  if (tp.ignore_z_rot) tol = 2.0f * tol;
  const float tc[4] = {-trot[0], -trot[1], -trot[2], trot[3]};
  float qd[4];
  t_quat_mul(orot, tc, qd);
  float qn = sqrtf(qd[0] * qd[0] + qd[1] * qd[1] + qd[2] * qd[2]);
  qn = qn > 1.0f ? 1.0f : qn;
  const float rot_dist = 2.0f * asinf(qn);
  const float dist_rew = goal_dist * tp.dist_reward_scale;
  const float rot_rew = 1.0f / (fabsf(rot_dist) + tp.rot_eps) * tp.rot_reward_scale;
  float pen = 0.0f;
  for (int i = 0; i < tp.num_actions; i++) pen += act[i] * act[i];
  float reward = dist_rew + rot_rew + pen * tp.action_penalty_scale;
  const int64_t goal_resets = fabsf(rot_dist) <= tol ? 1 : goal_in;
  const float succ = *successes + (float)goal_resets;
  if (goal_resets == 1) reward = reward + tp.reach_goal_bonus;
  if (goal_dist >= tp.fall_dist) reward = reward + tp.fall_penalty;
  int64_t resets = goal_dist >= tp.fall_dist ? 1 : reset_in;
  int64_t prog = *progress;
  if (tp.max_consecutive_successes > 0) {
    if (fabsf(rot_dist) <= tol) prog = 0;
    if (succ >= (float)tp.max_consecutive_successes) resets = 1;
  }
  if ((float)prog >= max_episode_length - 1.0f) resets = 1;
  if (tp.max_consecutive_successes > 0 && (float)prog >= max_episode_length - 1.0f)
    reward = reward + 0.5f * tp.fall_penalty;
  *rew = reward;
  *reset_out = resets;
  *goal_out = goal_resets;
  *progress = prog;
  *successes = succ;
}

// action -> PD target of DOF d (shadow_hand.py:677-693); returns the new target
__device__ __forceinline__ float h_target(const mg_task_params& tp, int d, float a, float prev) {
  const float lo = tp.dof_lower[d], hi = tp.dof_upper[d];
  float t;
  if (tp.use_relative_control) {
    t = prev + (float)((double)tp.dof_speed_scale * (double)tp.dt) * a;
  } else {
    t = 0.5f * (a + 1.0f) * (hi - lo) + lo;
    t = tp.act_moving_average * t + (1.0f - tp.act_moving_average) * prev;
  }
  t = t < hi ? t : hi;
  t = t > lo ? t : lo;
  return t;
}

// running mean of consecutive successes (shadow_hand.py:795-798)
__device__ __forceinline__ float h_cons_update(const mg_task_params& tp, int64_t num_resets, float finished,
                                               float cons) {
  if (num_resets > 0) return tp.av_factor * finished / (float)num_resets + (1.0f - tp.av_factor) * cons;
  return cons;
}

}  // namespace mg
