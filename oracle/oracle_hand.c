/*
 * oracle_hand.c — CPU restatement of the reference's in-hand manipulation task
 * layer (ShadowHand).  TEST INFRASTRUCTURE
 * ONLY (tests/, smoke(), bench.py cpu_baseline).
 *
 * PINNED against the reference's own outputs: tests/golden/jit_shadowhand.npz
 * (compute_hand_reward, randomize_rotation) and trace_shadowhand.npz (the whole
 * physics-free VecTask.step of tasks/shadow_hand.py on a fake gym), both made
 * by running the reference (tests/golden/make_golden.py, make_traces.py).
 * fp32 in the reference's operation order, built with -ffp-contract=off.
 *
 * Restated functions (reference file:line):
 *   quat_from_angle_axis / quat_unit / quat_conjugate   utils/torch_jit_utils.py:107-123
 *   scale / tensor_clamp / unscale                      utils/torch_jit_utils.py:229-240
 *   randomize_rotation                                  tasks/shadow_hand.py:803-806
 *   compute_hand_reward (incl. the global running mean) tasks/shadow_hand.py:746-800
 *   compute_full_state / compute_full_observations /
 *   compute_fingertip_observations (observationType)    tasks/shadow_hand.py:473-584
 *   reset_target_pose / reset_idx                       tasks/shadow_hand.py:586-668
 *   pre_physics_step (goal/env resets, PD targets)      tasks/shadow_hand.py:670-698
 *   post_physics_step + VecTask.step tail               tasks/shadow_hand.py:710-716,
 *                                                       tasks/base/vec_task.py:393-410
 */
#include <math.h>
#include <string.h>

#include "oracle.h"

#define PI_F 3.14159265358979323846f
/* injected noise row: [goal-only 4 | reset_idx 53 | reset_target_pose 4 | force prob 1 | force select 1 |
 * force direction 3] (shadow_hand.py:587, 610, 642-643, 704-706) */
#define HN_COLS 66
#define HN_FORCE_PROB 61
#define HN_FORCE_SEL 62
#define HN_FORCE_DIR 63

static void h_quat_mul(const float* a, const float* b, float* o) { /* torch_jit_utils.py:41-62 */
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

/* quat_from_angle_axis(angle, unit axis e_k) */
static void h_quat_from_angle_axis(float angle, int k, float* q) {
  float theta = angle / 2.0f;
  float s = sinf(theta), c = cosf(theta);
  float v[4] = {0.0f, 0.0f, 0.0f, c};
  v[k] = 1.0f * s;
  float n = sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3]);
  n = n < 1e-9f ? 1e-9f : n;
  for (int i = 0; i < 4; i++) q[i] = v[i] / n;
}

void orc_randomize_rotation(float r0, float r1, float* q) {
  float qa[4], qb[4];
  h_quat_from_angle_axis(r0 * PI_F, 0, qa);
  h_quat_from_angle_axis(r1 * PI_F, 1, qb);
  h_quat_mul(qa, qb, q);
}

/* randomize_rotation_pen(rand0, rand1, max_angle = tensor(0.3), x, y, z) (shadow_hand.py:810-813): rand1 is
 * unused, as in the reference */
static void randomize_rotation_pen(float r0, float* q) {
  float qa[4], qb[4];
  h_quat_from_angle_axis((float)(0.5 * 3.14159265358979323846) + r0 * 0.3f, 0, qa);
  h_quat_from_angle_axis(r0 * PI_F, 2, qb);
  h_quat_mul(qa, qb, q);
}

/* the object's reset orientation (shadow_hand.py:625-629): pen (ignore_z_rot) or generic */
static void object_reset_rotation(const mg_task_params* tp, float r0, float r1, float* q) {
  if (tp->ignore_z_rot) randomize_rotation_pen(r0, q);
  else orc_randomize_rotation(r0, r1, q);
}

/* per-env part of compute_hand_reward; returns the updated successes etc. through pointers */
static void hand_reward_one(const mg_task_params* tp, float max_episode_length, const float* opos, const float* orot,
                            const float* tpos, const float* trot, const float* act, int64_t reset_in,
                            int64_t goal_in, int64_t* progress, float* successes, float* rew, int64_t* reset_out,
                            int64_t* goal_out) {
  float d0 = opos[0] - tpos[0], d1 = opos[1] - tpos[1], d2 = opos[2] - tpos[2];
  float goal_dist = sqrtf(d0 * d0 + d1 * d1 + d2 * d2);
  float tol = tp->success_tolerance;
  if (tp->ignore_z_rot) tol = 2.0f * tol;
  float tc[4] = {-trot[0], -trot[1], -trot[2], trot[3]}, qd[4];
  h_quat_mul(orot, tc, qd);
  float qn = sqrtf(qd[0] * qd[0] + qd[1] * qd[1] + qd[2] * qd[2]);
  qn = qn > 1.0f ? 1.0f : qn;
  float rot_dist = 2.0f * asinf(qn);
  float dist_rew = goal_dist * tp->dist_reward_scale;
  float rot_rew = 1.0f / (fabsf(rot_dist) + tp->rot_eps) * tp->rot_reward_scale;
  float pen = 0.0f;
  for (int i = 0; i < tp->num_actions; i++) pen += act[i] * act[i];
  float reward = dist_rew + rot_rew + pen * tp->action_penalty_scale;
  int64_t goal_resets = fabsf(rot_dist) <= tol ? 1 : goal_in;
  float succ = *successes + (float)goal_resets;
  if (goal_resets == 1) reward = reward + tp->reach_goal_bonus;
  if (goal_dist >= tp->fall_dist) reward = reward + tp->fall_penalty;
  int64_t resets = goal_dist >= tp->fall_dist ? 1 : reset_in;
  int64_t prog = *progress;
  if (tp->max_consecutive_successes > 0) {
    if (fabsf(rot_dist) <= tol) prog = 0;
    if (succ >= (float)tp->max_consecutive_successes) resets = 1;
  }
  if ((float)prog >= max_episode_length - 1.0f) resets = 1;
  if (tp->max_consecutive_successes > 0 && (float)prog >= max_episode_length - 1.0f)
    reward = reward + 0.5f * tp->fall_penalty;
  *rew = reward;
  *reset_out = resets;
  *goal_out = goal_resets;
  *progress = prog;
  *successes = succ;
}

/* running mean of consecutive successes over the envs that reset (shadow_hand.py:795-798) */
static float hand_cons_update(const mg_task_params* tp, int64_t num_resets, float finished, float cons) {
  if (num_resets > 0) return tp->av_factor * finished / (float)num_resets + (1.0f - tp->av_factor) * cons;
  return cons;
}

int orc_hand_reward(const mg_task_params* tp, int32_t n, float max_episode_length, const float* object_pos,
                    const float* object_rot, const float* target_pos, const float* target_rot, const float* actions,
                    int64_t* reset, int64_t* reset_goal, int64_t* progress, float* successes, float* cons,
                    float* rew) {
  int64_t nres = 0;
  float fin = 0.0f;
  for (int e = 0; e < n; e++) {
    int64_t ro, go;
    hand_reward_one(tp, max_episode_length, object_pos + 3 * e, object_rot + 4 * e, target_pos + 3 * e,
                    target_rot + 4 * e, actions + (size_t)tp->num_actions * e, reset[e], reset_goal[e], progress + e,
                    successes + e, rew + e, &ro, &go);
    reset[e] = ro;
    reset_goal[e] = go;
    nres += ro;
    fin += successes[e] * (float)ro;
  }
  *cons = hand_cons_update(tp, nres, fin, *cons);
  return 0;
}

/* ---------------------------------------------------------------- resets + targets */
static float hu(const mg_task_buffers* tb, int e, int k) {
  return tb->noise ? tb->noise[(size_t)HN_COLS * e + k]
                   : orc_uniform(tb->seed, (uint64_t)(tb->env_offset + e), tb->step_counter, (uint32_t)k);
}
static float rand_pm1(float u) { return 2.0f * u + -1.0f; } /* torch_rand_float(-1, 1): (1 - -1) * u + -1 */

/* N(0,1) draw k: injected column, or Box-Muller on two counter-based uniforms (same recipe as the GPU) */
static float hn(const mg_task_buffers* tb, int e, int k) {
  if (tb->noise) return tb->noise[(size_t)HN_COLS * e + k];
  const uint64_t gid = (uint64_t)(tb->env_offset + e);
  const float u1 = orc_uniform(tb->seed, gid, tb->step_counter, (uint32_t)(128 + 2 * k));
  const float u2 = orc_uniform(tb->seed, gid, tb->step_counter, (uint32_t)(129 + 2 * k));
  return sqrtf(-2.0f * logf(1.0f - u1)) * cosf(6.28318530717958647f * u2);
}

/* random object force of env e (shadow_hand.py:641-643 reset_idx; 700-706 pre_physics_step):
 * a reset zeroes rb_forces[e] and redraws random_force_prob[e] = exp((log lo - log hi) u + log hi);
 * with forceScale > 0 the force decays by forceDecay^(dt/forceDecayInterval) and, when
 * U(0,1) < prob, becomes randn(3) * object mass * forceScale. */
static void object_force(const mg_task_params* tp, const mg_task_buffers* tb, int e, int env_reset, float* f) {
  float prob = tb->random_force_prob ? tb->random_force_prob[e] : 0.0f;
  if (env_reset) {
    f[0] = f[1] = f[2] = 0.0f;
    const float lhi = logf(tp->force_prob_hi);
    prob = expf((logf(tp->force_prob_lo) - lhi) * hu(tb, e, HN_FORCE_PROB) + lhi);
    if (tb->random_force_prob) tb->random_force_prob[e] = prob;
  }
  if (tp->force_scale > 0.0f) {
    for (int k = 0; k < 3; k++) f[k] = f[k] * tp->force_decay_step;
    if (hu(tb, e, HN_FORCE_SEL) < prob)
      for (int k = 0; k < 3; k++) f[k] = hn(tb, e, HN_FORCE_DIR + k) * tp->object_rb_mass * tp->force_scale;
  }
}

static void reset_target_pose(const mg_task_params* tp, const mg_task_buffers* tb, float* root_env, int e,
                              float g0, float g1) {
  float q[4];
  orc_randomize_rotation(g0, g1, q);
  float* gs = tb->goal_states + 13 * (size_t)e;
  gs[0] = tp->object_start[0];
  gs[1] = tp->object_start[1];
  gs[2] = tp->object_start[2] + tp->goal_dz;
  for (int k = 0; k < 4; k++) gs[3 + k] = q[k];
  float* gr = root_env + 26;
  for (int k = 0; k < 3; k++) gr[k] = gs[k] + tp->goal_displacement[k];
  for (int k = 0; k < 4; k++) gr[3 + k] = q[k];
  for (int k = 7; k < 13; k++) gr[k] = 0.0f;
  tb->reset_goal[e] = 0;
}

int orc_hand_pre_physics(const mg_model* m, const mg_task_params* tp, const mg_state_views* v,
                         const mg_task_buffers* tb, int32_t n) {
  const int nd = m->num_dofs, na = tp->num_actions;
  float* tgt = (float*)v->dof_targets;
  for (int e = 0; e < n; e++) {
    float* root = v->root_states + (size_t)39 * e;
    const int goal_only = tb->reset_goal[e] != 0, env_reset = tb->reset[e] != 0;
    if (goal_only) reset_target_pose(tp, tb, root, e, rand_pm1(hu(tb, e, 0)), rand_pm1(hu(tb, e, 1)));
    if (env_reset) {
      float r[53];
      for (int k = 0; k < 53; k++) r[k] = rand_pm1(hu(tb, e, 4 + k));
      reset_target_pose(tp, tb, root, e, rand_pm1(hu(tb, e, 57)), rand_pm1(hu(tb, e, 58)));
      float* ob = root + 13;
      ob[0] = tp->object_start[0] + tp->reset_position_noise * r[0];
      ob[1] = tp->object_start[1] + tp->reset_position_noise * r[1];
      ob[2] = tp->object_start[2] + tp->reset_position_noise * r[2];
      object_reset_rotation(tp, r[3], r[4], ob + 3);
      for (int k = 7; k < 13; k++) ob[k] = 0.0f;
      float* dof = v->dof_state + (size_t)2 * nd * e;
      for (int j = 0; j < nd; j++) {
        float dmax = tp->dof_upper[j] - tp->initial_dof_pos[j], dmin = tp->dof_lower[j] - tp->initial_dof_pos[j];
        float rd = dmin + (dmax - dmin) * 0.5f * (r[5 + j] + 1.0f);
        float pos = tp->initial_dof_pos[j] + tp->reset_dof_pos_noise * rd;
        dof[2 * j] = pos;
        dof[2 * j + 1] = 0.0f + tp->reset_dof_vel_noise * r[5 + nd + j];
        tb->prev_targets[(size_t)nd * e + j] = pos;
        tgt[(size_t)nd * e + j] = pos;
      }
      tb->progress[e] = 0;
      tb->reset[e] = 0;
      tb->successes[e] = 0.0f;
    }
    /* actions -> PD targets (shadow_hand.py:677-693) */
    for (int i = 0; i < na; i++) {
      const int d = tp->actuated_dof[i];
      float a = tb->actions[(size_t)na * e + i];
      a = a < tp->clip_actions ? a : tp->clip_actions;
      a = a > -tp->clip_actions ? a : -tp->clip_actions;
      if (tb->actions_out) tb->actions_out[(size_t)na * e + i] = a;
      const float lo = tp->dof_lower[d], hi = tp->dof_upper[d];
      float* prev = tb->prev_targets + (size_t)nd * e + d;
      float t;
      if (tp->use_relative_control) {
        t = *prev + (float)((double)tp->dof_speed_scale * (double)tp->dt) * a;
      } else {
        t = 0.5f * (a + 1.0f) * (hi - lo) + lo;
        t = tp->act_moving_average * t + (1.0f - tp->act_moving_average) * *prev;
      }
      t = t < hi ? t : hi;
      t = t > lo ? t : lo;
      tgt[(size_t)nd * e + d] = t;
      *prev = t;
    }
    if (v->rb_forces || tb->random_force_prob) {
      float* fr = v->rb_forces ? v->rb_forces + ((size_t)tp->rb_per_env * e + tp->object_rb) * 3 : NULL;
      float f[3] = {fr ? fr[0] : 0.0f, fr ? fr[1] : 0.0f, fr ? fr[2] : 0.0f};
      object_force(tp, tb, e, env_reset, f);
      if (fr)
        for (int k = 0; k < 3; k++) fr[k] = f[k];
    }
  }
  return 0;
}

/* ---------------------------------------------------------------- observations */
/* observationType layouts (shadow_hand.py:473-584): compute_full_state (211),
 * compute_full_observations (157; no_vel: 77), compute_fingertip_observations(no_vel) (42) */
enum { DOFP, DOFV, DOFF, OPOSE, OPOS, OLIN, OANG, GPOSE, QDIFF, FTS, FTP, FTF, ACTS, END };
static const int LAYOUT[4][12] = {
    {DOFP, DOFV, DOFF, OPOSE, OLIN, OANG, GPOSE, QDIFF, FTS, FTF, ACTS, END},
    {DOFP, DOFV, OPOSE, OLIN, OANG, GPOSE, QDIFF, FTS, ACTS, END, END, END},
    {DOFP, OPOSE, GPOSE, QDIFF, FTP, ACTS, END, END, END, END, END, END},
    {FTP, OPOS, QDIFF, ACTS, END, END, END, END, END, END, END, END}};

static void hand_obs_one(int layout, const mg_model* m, const mg_task_params* tp, const mg_state_views* v,
                         const mg_task_buffers* tb, const float* act, int e, float* o) {
  const int nd = m->num_dofs, nb = tp->rb_per_env, nf = tp->num_fingertips;
  const float* dof = v->dof_state + (size_t)2 * nd * e;
  const float* ob = v->root_states + (size_t)39 * e + 13;
  const float* gs = tb->goal_states + (size_t)13 * e;
  const float* rbs = v->rigid_body_states + (size_t)13 * nb * e;
  float gc[4] = {-gs[3], -gs[4], -gs[5], gs[6]}, qdiff[4];
  h_quat_mul(ob + 3, gc, qdiff);
  int k = 0;
  for (int s = 0; s < 12 && LAYOUT[layout & 3][s] != END; s++) {
    switch (LAYOUT[layout & 3][s]) {
      case DOFP:
        for (int j = 0; j < nd; j++)
          o[k++] = (2.0f * dof[2 * j] - tp->dof_upper[j] - tp->dof_lower[j]) / (tp->dof_upper[j] - tp->dof_lower[j]);
        break;
      case DOFV: for (int j = 0; j < nd; j++) o[k++] = tp->vel_obs_scale * dof[2 * j + 1]; break;
      case DOFF: for (int j = 0; j < nd; j++) o[k++] = tp->force_torque_obs_scale * v->dof_force[(size_t)nd * e + j]; break;
      case OPOSE: for (int c = 0; c < 7; c++) o[k++] = ob[c]; break;
      case OPOS: for (int c = 0; c < 3; c++) o[k++] = ob[c]; break;
      case OLIN: for (int c = 7; c < 10; c++) o[k++] = ob[c]; break;
      case OANG: for (int c = 10; c < 13; c++) o[k++] = tp->vel_obs_scale * ob[c]; break;
      case GPOSE: for (int c = 0; c < 7; c++) o[k++] = gs[c]; break;
      case QDIFF: for (int c = 0; c < 4; c++) o[k++] = qdiff[c]; break;
      case FTS:
      case FTP: {
        const int w = LAYOUT[layout & 3][s] == FTS ? 13 : 3;
        for (int f = 0; f < nf; f++)
          for (int c = 0; c < w; c++) o[k++] = rbs[(size_t)13 * tp->fingertip_body[f] + c];
        break;
      }
      case FTF: for (int c = 0; c < 6 * nf; c++) o[k++] = tp->force_torque_obs_scale * v->sensors[(size_t)6 * nf * e + c]; break;
      case ACTS: for (int i = 0; i < tp->num_actions; i++) o[k++] = act[i]; break;
    }
  }
}

int orc_hand_post_physics(const mg_model* m, const mg_task_params* tp, const mg_state_views* v,
                          const mg_task_buffers* tb, int32_t n) {
  const int na = tp->num_actions, no = tp->num_obs;
  int64_t nres = 0;
  float fin = 0.0f;
  const float max_ep = (float)tp->max_episode_length;
  for (int e = 0; e < n; e++) {
    tb->progress[e] += 1;
    const float* act = tb->actions_out + (size_t)na * e;
    float* o = tb->obs + (size_t)no * e;
    hand_obs_one(tp->obs_type, m, tp, v, tb, act, e, o);
    /* asymmetric_observations: states_buf = compute_full_state(asymm_obs=True) (shadow_hand.py:470-471) */
    if (tb->states && tp->num_states > 0) hand_obs_one(0, m, tp, v, tb, act, e, tb->states + (size_t)tp->num_states * e);
    const float* ob = v->root_states + (size_t)39 * e + 13;
    const float* gs = tb->goal_states + (size_t)13 * e;
    int64_t ro, go;
    hand_reward_one(tp, max_ep, ob, ob + 3, gs, gs + 3, act, tb->reset[e], tb->reset_goal[e], tb->progress + e,
                    tb->successes + e, tb->rew + e, &ro, &go);
    tb->reset[e] = ro;
    tb->reset_goal[e] = go;
    nres += ro;
    fin += tb->successes[e] * (float)ro;
    tb->timeout[e] = (uint8_t)((tb->progress[e] >= (int64_t)tp->max_episode_length - 1) && (ro != 0));
    if (tb->obs_clamped)
      for (int i = 0; i < no; i++) {
        float x = o[i];
        x = x < tp->clip_obs ? x : tp->clip_obs;
        x = x > -tp->clip_obs ? x : -tp->clip_obs;
        tb->obs_clamped[(size_t)no * e + i] = x;
      }
  }
  if (tb->defer_finalize) {  /* partial sums for a cross-rank all-reduce (mg_hand_finalize) */
    tb->reduce_scratch[0] += (uint64_t)nres;
    tb->reduce_scratch[1] += (uint64_t)fin;
    return 0;
  }
  tb->consecutive_successes[0] = hand_cons_update(tp, nres, fin, tb->consecutive_successes[0]);
  return 0;
}

int orc_hand_finalize(const mg_task_params* tp, const mg_task_buffers* tb) {
  tb->consecutive_successes[0] =
      hand_cons_update(tp, (int64_t)tb->reduce_scratch[0], (float)tb->reduce_scratch[1], tb->consecutive_successes[0]);
  tb->reduce_scratch[0] = 0;
  tb->reduce_scratch[1] = 0;
  return 0;
}

int orc_hand_env_step(const mg_model* m, const mg_sim_params* p, const mg_task_params* tp,
                      const mg_state_views* v, const mg_task_buffers* tb, int32_t n, int32_t threads) {
  orc_hand_pre_physics(m, tp, v, tb, n);
  /* gym.simulate x controlFrequencyInv (vec_task.py:381-384) */
  for (int k = 0; k < (tp->control_freq_inv > 1 ? tp->control_freq_inv : 1); k++)
    orc_simulate_views(m, p, n, v, threads);
  return orc_hand_post_physics(m, tp, v, tb, n);
}
