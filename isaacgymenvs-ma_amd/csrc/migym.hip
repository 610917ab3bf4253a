// migym.hip — C-ABI (include/migym.h) and kernels of the MI355X physics-step +
// observation/reward path.  One lane per actor/env; every kernel is
// asynchronous on the caller's stream; no entry point synchronises.
#include <hip/hip_runtime.h>

#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "dispatch.hpp"
#include "hand_task.hpp"
#include "task.hpp"

namespace {
thread_local std::string g_err;
}  // namespace
int mgi::fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
using mgi::fail;
using mgi::kBlock;
namespace {
int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(MG_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
  return MG_OK;
}
inline int grid_for(int n) { return (n + kBlock - 1) / kBlock; }

// publish the phase-timing buffer to every instance's code object
template <int... I>
int publish_all(unsigned long long* buf, std::integer_sequence<int, I...>) {
  int rc = MG_OK;
  ((rc = rc ? rc : mgi::phase_buf_publish<I>(buf)), ...);
  return rc;
}
}  // namespace

__global__ __launch_bounds__(kBlock) void k_observations(mg_task_params tp, int n, const float* __restrict__ root,
                                                         const float* __restrict__ dof, const float* __restrict__ dforce,
                                                         const float* __restrict__ sensors,
                                                         const float* __restrict__ actions, float* pot, float* prev_pot,
                                                         float* up, float* heading, float* obs) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const int nd = mg::t_dofs(&tp), ns = mg::t_sensors(&tp);
  const float zero3[3] = {0.0f, 0.0f, 0.0f};
  mg::obs_env(&tp, zero3, root + (size_t)13 * e, dof + (size_t)2 * nd * e, dforce ? dforce + (size_t)nd * e : nullptr,
              sensors ? sensors + (size_t)6 * ns * e : nullptr, actions + (size_t)tp.num_actions * e, pot + e,
              prev_pot + e, up + 3 * (size_t)e, heading + 3 * (size_t)e, obs + (size_t)tp.num_obs * e);
}

__global__ __launch_bounds__(kBlock) void k_reward(mg_task_params tp, int n, const float* __restrict__ obs,
                                                   const float* __restrict__ actions, const float* __restrict__ pot,
                                                   const float* __restrict__ prev_pot,
                                                   const int64_t* __restrict__ progress, int64_t* reset, float* rew) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  mg::reward_env(&tp, obs + (size_t)tp.num_obs * e, actions + (size_t)tp.num_actions * e, pot[e], prev_pot[e],
                 progress[e], reset + e, rew + e);
}

// post_physics_step + VecTask.step tail for actor a (state already advanced).  Multi-agent:
// actors of one env are adjacent lanes of one wave (64 % num_agents == 0), so the env-level
// AND of the agents' reset flags is a ballot and the other agents' torso positions are shuffles.
__device__ __forceinline__ void post_physics_env(const mg_task_params& tp, const mg_state_views& v,
                                                 const mg_task_buffers& tb, int a, const float* act,
                                                 int64_t reset_in) {
  const int nd = mg::t_dofs(&tp), ns = mg::t_sensors(&tp), no = tp.num_obs;
  const int A = tp.num_agents > 1 ? tp.num_agents : 1;
  const int k = a % A;
  const float* off = tp.agent_offset[k];
  float* root = v.root_states + (size_t)13 * a;
  float* dof = v.dof_state + (size_t)2 * nd * a;
  int64_t progress = tb.progress[a] + 1;
  int64_t reset = reset_in;
  bool do_reset = reset != 0;
  if (A > 1) {  // AND filter (franka_reach_MA.py:875-885)
    const int lane = threadIdx.x & 63;
    const unsigned long long m = __ballot(reset != 0);
    const unsigned long long full = (A >= 64) ? ~0ull : ((1ull << A) - 1ull);
    do_reset = ((m >> (lane - k)) & full) == full;
  }
  float pot = tb.potentials ? tb.potentials[a] : 0.0f;
  float prev = tb.prev_potentials ? tb.prev_potentials[a] : 0.0f;
  if (do_reset) {
    mg::reset_env(&tp, off, tb.noise ? tb.noise + (size_t)2 * nd * a : nullptr, tb.seed,
                  (uint64_t)(tb.env_offset * A + a), tb.step_counter, root, dof, &pot, &prev);
    progress = 0;
    reset = 0;
  }
  float* o = tb.obs + (size_t)no * a;
  float up[3], hd[3];
  mg::obs_env(&tp, off, root, dof, v.dof_force ? v.dof_force + (size_t)nd * a : nullptr,
              v.sensors ? v.sensors + (size_t)6 * ns * a : nullptr, act, &pot, &prev, up, hd, o);
  if (A > 1) {  // "others" block: cyclic shift starting after self (franka_reach_MA.py:604-608)
    const int lane = threadIdx.x & 63;
    const float px = root[0], py = root[1], pz = root[2];
    const int base = no - 3 * (A - 1);
    for (int j = 1; j < A; j++) {
      const int src = lane - k + (k + j) % A;
      const float qx = __shfl(px, src), qy = __shfl(py, src), qz = __shfl(pz, src);
      o[base + 3 * (j - 1) + 0] = qx - px;
      o[base + 3 * (j - 1) + 1] = qy - py;
      o[base + 3 * (j - 1) + 2] = qz - pz;
    }
  }
  float rew;
  mg::reward_env(&tp, o, act, pot, prev, progress, &reset, &rew);
  const float max_ep_m1 = (float)tp.max_episode_length - 1.0f;
  tb.rew[a] = rew;
  tb.reset[a] = reset;
  tb.progress[a] = progress;
  tb.timeout[a] = (uint8_t)(((float)progress >= max_ep_m1) && (reset != 0));
  if (tp.task_id != MG_TASK_CARTPOLE) {
    tb.potentials[a] = pot;
    tb.prev_potentials[a] = prev;
    for (int c = 0; c < 3; c++) {
      tb.up_vec[3 * (size_t)a + c] = up[c];
      tb.heading_vec[3 * (size_t)a + c] = hd[c];
    }
  }
  if (tb.obs_clamped)
    for (int i = 0; i < no; i++) tb.obs_clamped[(size_t)no * a + i] = mg::clampf(o[i], tp.clip_obs);
  if (tb.out_pack) {  // the gather's message row [clamped obs | rew | reset]
    float* pk = tb.out_pack + (size_t)(no + 2) * a;
    for (int i = 0; i < no; i++) pk[i] = mg::clampf(o[i], tp.clip_obs);
    pk[no] = rew;
    pk[no + 1] = (float)reset;
  }
}

__global__ __launch_bounds__(kBlock) void k_post_physics(mg_task_params tp, mg_state_views v, mg_task_buffers tb,
                                                         int n) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const int na = tp.num_actions;
  float act[64];
  for (int i = 0; i < na; i++) {
    act[i] = mg::clampf(tb.actions[(size_t)na * e + i], tp.clip_actions);
    if (tb.actions_out) tb.actions_out[(size_t)na * e + i] = act[i];
  }
  post_physics_env(tp, v, tb, e, act, tb.reset[e]);
}


// pre_physics_step of the locomotion tasks: effort = clamp(a) * gear * power_scale
// (ant.py:281-285, humanoid.py:281-285; cartpole.py:159-163: DOF 0 only)
__global__ __launch_bounds__(kBlock) void k_pre_loco(mg_task_params tp, mg_state_views v, mg_task_buffers tb, int n,
                                                     int nd) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * nd) return;
  const int a = t / nd, d = t % nd, na = tp.num_actions;
  float tau;
  if (tp.task_id == MG_TASK_CARTPOLE) {
    tau = d == 0 ? mg::clampf(tb.actions[(size_t)na * a], tp.clip_actions) * tp.power_scale : 0.0f;
  } else {
    const float act = d < na ? mg::clampf(tb.actions[(size_t)na * a + d], tp.clip_actions) : 0.0f;
    tau = act * tp.motor_effort[d] * tp.power_scale;
  }
  const_cast<float*>(v.dof_actuation)[t] = tau;
}


// reset_idx of one ShadowHand env on one lane (shadow_hand.py:586-668): goal (reset_target_pose), object
// pose, hand DOFs and PD targets, counters
__device__ void hand_reset_env(const mg_task_params& tp, const mg_state_views& v, const mg_task_buffers& tb, int e,
                               int nd, uint64_t gid) {
  float* root = v.root_states + (size_t)39 * e;
  float* gs = tb.goal_states + (size_t)13 * e;
  float* tgt = const_cast<float*>(v.dof_targets) + (size_t)nd * e;
  float* prev = tb.prev_targets + (size_t)nd * e;
  {
    mg::h_reset_goal(tp, mg::h_rand_pm1(mg::h_uniform(tb, e, gid, 57)),
                     mg::h_rand_pm1(mg::h_uniform(tb, e, gid, 58)), gs, root + 26);
    float r[5];
    for (int k = 0; k < 5; k++) r[k] = mg::h_rand_pm1(mg::h_uniform(tb, e, gid, 4 + k));
    float* ob = root + 13;
    for (int k = 0; k < 3; k++) ob[k] = tp.object_start[k] + tp.reset_position_noise * r[k];
    mg::h_object_reset_rotation(tp, r[3], r[4], ob + 3);
    for (int k = 7; k < 13; k++) ob[k] = 0.0f;
    float* dof = v.dof_state + (size_t)2 * nd * e;
    for (int j = 0; j < nd; j++) {
      const float rp = mg::h_rand_pm1(mg::h_uniform(tb, e, gid, 9 + j));
      const float rv = mg::h_rand_pm1(mg::h_uniform(tb, e, gid, 9 + nd + j));
      const float dmax = tp.dof_upper[j] - tp.initial_dof_pos[j], dmin = tp.dof_lower[j] - tp.initial_dof_pos[j];
      const float pos = tp.initial_dof_pos[j] + tp.reset_dof_pos_noise * (dmin + (dmax - dmin) * 0.5f * (rp + 1.0f));
      dof[2 * j] = pos;
      dof[2 * j + 1] = 0.0f + tp.reset_dof_vel_noise * rv;
      prev[j] = pos;
      tgt[j] = pos;
    }
    tb.progress[e] = 0;
    tb.reset[e] = 0;
    tb.successes[e] = 0.0f;
  }
}

// reset_idx(ids) of the locomotion tasks, one lane per listed actor (ant.py:252-279): DOF noise, root row
// and potentials from task.hpp's reset_dof / reset_root (the fused step's own reset code), counters cleared
__global__ __launch_bounds__(kBlock) void k_reset_idx(mg_task_params tp, mg_state_views v, mg_task_buffers tb,
                                                      const int32_t* ids, int n, int n_actors) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int a = ids[t];
  if (a < 0 || a >= n_actors) return;
  if (tp.task_id == MG_TASK_SHADOW_HAND) {
    const uint64_t gid = (uint64_t)(tb.env_offset + a);
    hand_reset_env(tp, v, tb, a, tp.num_dofs, gid);
    tb.reset_goal[a] = 0;
    // random object forces: reset_idx zeroes the force and redraws the env's probability (shadow_hand.py:641-643)
    if (tb.random_force_prob) {
      const float lhi = logf(tp.force_prob_hi);
      tb.random_force_prob[a] = expf((logf(tp.force_prob_lo) - lhi) * mg::h_uniform(tb, a, gid, mg::HN_FORCE_PROB) + lhi);
    }
    if (v.rb_forces)
      for (int k = 0; k < 3; k++) v.rb_forces[((size_t)tp.rb_per_env * a + tp.rb_per_env - 2) * 3 + k] = 0.0f;
    return;
  }
  const int A = tp.num_agents > 1 ? tp.num_agents : 1;
  const int nd = mg::t_dofs(&tp);
  const float* nz = tb.noise ? tb.noise + (size_t)2 * nd * a : nullptr;
  float* dof = v.dof_state + (size_t)2 * nd * a;
  for (int i = 0; i < nd; i++)
    mg::reset_dof(&tp, i, nd, nz, tb.seed, (uint64_t)(tb.env_offset * A + a), tb.step_counter, dof);
  float pot = 0.0f, prev = 0.0f;
  mg::reset_root(&tp, tp.agent_offset[a % A], v.root_states + (size_t)13 * a, &pot, &prev);
  if (tp.task_id != MG_TASK_CARTPOLE && tb.potentials) {
    tb.potentials[a] = pot;
    tb.prev_potentials[a] = prev;
  }
  tb.progress[a] = 0;
  tb.reset[a] = 0;
}

// pre_physics_step of one env on one lane (physics-free path, shadow_hand.py:670-698)
__global__ __launch_bounds__(kBlock) void k_hand_pre(mg_task_params tp, mg_state_views v, mg_task_buffers tb,
                                                     int n, int nd) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const uint64_t gid = (uint64_t)(tb.env_offset + e);
  float* root = v.root_states + (size_t)39 * e;
  float* gs = tb.goal_states + (size_t)13 * e;
  const bool goal_reset = tb.reset_goal[e] != 0, env_reset = tb.reset[e] != 0;
  if (goal_reset)
    mg::h_reset_goal(tp, mg::h_rand_pm1(mg::h_uniform(tb, e, gid, 0)), mg::h_rand_pm1(mg::h_uniform(tb, e, gid, 1)),
                     gs, root + 26);
  float* tgt = const_cast<float*>(v.dof_targets) + (size_t)nd * e;
  float* prev = tb.prev_targets + (size_t)nd * e;
  if (env_reset) hand_reset_env(tp, v, tb, e, nd, gid);
  if (goal_reset || env_reset) tb.reset_goal[e] = 0;
  const int na = tp.num_actions;
  for (int i = 0; i < na; i++) {
    const int d = tp.actuated_dof[i];
    const float a = mg::clampf(tb.actions[(size_t)na * e + i], tp.clip_actions);
    if (tb.actions_out) tb.actions_out[(size_t)na * e + i] = a;
    const float t = mg::h_target(tp, d, a, prev[d]);
    tgt[d] = t;
    prev[d] = t;
  }
  // random object forces (reset_idx's zeroing + probability redraw, then decay / new draws)
  if (v.rb_forces || tb.random_force_prob) {
    float* fr = v.rb_forces ? v.rb_forces + ((size_t)tp.rb_per_env * e + tp.object_rb) * 3 : nullptr;
    float f[3] = {fr ? fr[0] : 0.0f, fr ? fr[1] : 0.0f, fr ? fr[2] : 0.0f};
    mg::h_object_force(tp, tb, e, gid, env_reset, f);
    if (fr)
      for (int k = 0; k < 3; k++) fr[k] = f[k];
  }
}

// observation value k of one env from its state rows (observationType layout, hand_task.hpp)
__device__ __forceinline__ float hand_obs_value(int layout, const mg_task_params& tp, int k, int nd, const float* dof,
                                                const float* dforce, const float* orow, const float* gs,
                                                const float* qdiff, const float* rbs, const float* sens,
                                                const float* act) {
  int i;
  const int seg = mg::h_locate_in(layout, tp, nd, k, &i);
  if (seg == mg::HS_FT_STATE || seg == mg::HS_FT_POS) {
    int b, c;
    mg::h_ft_ref(tp, seg, i, &b, &c);
    return rbs[(size_t)13 * b + c];
  }
  return mg::h_obs_value(tp, seg, i, dof, dforce, orow, gs, qdiff, sens, act);
}

// post_physics_step of one env on one lane (physics-free path): progress, full_state obs, reward,
// the running-mean partial sums, timeout, obs clamp
__global__ __launch_bounds__(kBlock) void k_hand_post(mg_task_params tp, mg_state_views v, mg_task_buffers tb,
                                                      int n, int nd) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  int64_t ro = 0;
  float fin = 0.0f;
  if (e < n) {
    const int na = tp.num_actions, no = tp.num_obs;
    const float* orow = v.root_states + (size_t)39 * e + 13;
    const float* gs = tb.goal_states + (size_t)13 * e;
    const float* act = tb.actions_out + (size_t)na * e;
    float qdiff[4];
    const float gc[4] = {-gs[3], -gs[4], -gs[5], gs[6]};
    mg::t_quat_mul(orow + 3, gc, qdiff);
    int64_t prog = tb.progress[e] + 1;
    float* o = tb.obs + (size_t)no * e;
    const float* rbs = v.rigid_body_states + (size_t)13 * tp.rb_per_env * e;
    for (int k = 0; k < no; k++) {
      const float x = hand_obs_value(tp.obs_type, tp, k, nd, v.dof_state + (size_t)2 * nd * e,
                                     v.dof_force + (size_t)nd * e, orow, gs, qdiff, rbs,
                                     v.sensors + (size_t)6 * tp.num_fingertips * e, act);
      o[k] = x;
      if (tb.obs_clamped) tb.obs_clamped[(size_t)no * e + k] = mg::clampf(x, tp.clip_obs);
    }
    if (tb.states)  // asymmetric_observations: states_buf = compute_full_state(asymm_obs=True)
      for (int k = 0; k < tp.num_states; k++)
        tb.states[(size_t)tp.num_states * e + k] =
            hand_obs_value(0, tp, k, nd, v.dof_state + (size_t)2 * nd * e, v.dof_force + (size_t)nd * e, orow, gs,
                           qdiff, rbs, v.sensors + (size_t)6 * tp.num_fingertips * e, act);
    float succ = tb.successes[e], rew;
    int64_t go;
    mg::h_reward(tp, orow, orow + 3, gs, gs + 3, act, tb.reset[e], tb.reset_goal[e], &prog, &succ, &rew, &ro, &go);
    tb.rew[e] = rew;
    tb.reset[e] = ro;
    tb.reset_goal[e] = go;
    tb.progress[e] = prog;
    tb.successes[e] = succ;
    tb.timeout[e] = (uint8_t)((prog >= (int64_t)tp.max_episode_length - 1) && (ro != 0));
    fin = succ * (float)ro;
    if (tb.out_pack) {  // the gather's message row [clamped obs | rew | reset]
      float* pk = tb.out_pack + (size_t)(no + 2) * e;
      for (int k = 0; k < no; k++) pk[k] = mg::clampf(o[k], tp.clip_obs);
      pk[no] = rew;
      pk[no + 1] = (float)ro;
    }
  }
  // partial sums of compute_hand_reward's global reduction (integer-valued: exact in any order)
  unsigned long long cr = (unsigned long long)ro, cf = (unsigned long long)fin;
  for (int off = 32; off >= 1; off >>= 1) {
    cr += __shfl_xor(cr, off);
    cf += __shfl_xor(cf, off);
  }
  if ((threadIdx.x & 63) == 0 && (cr | cf)) {
    atomicAdd((unsigned long long*)&tb.reduce_scratch[0], cr);
    atomicAdd((unsigned long long*)&tb.reduce_scratch[1], cf);
  }
}

// consecutive_successes running mean (shadow_hand.py:795-798) from the step's sums; clears them
__global__ void k_hand_finalize(mg_task_params tp, mg_task_buffers tb) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const int64_t nres = (int64_t)tb.reduce_scratch[0];
  const float fin = (float)tb.reduce_scratch[1];
  tb.consecutive_successes[0] = mg::h_cons_update(tp, nres, fin, tb.consecutive_successes[0]);
  tb.reduce_scratch[0] = 0;
  tb.reduce_scratch[1] = 0;
}


__global__ void k_set_indexed(float* __restrict__ dst, const float* __restrict__ src, const int32_t* __restrict__ idx,
                              int nidx, int row, int div) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nidx * row) return;
  const int r = t / row, c = t % row;
  const size_t a = (size_t)(idx[r] / div) * row + c;
  dst[a] = src[a];
}

// ------------------------------------------------------------------------------------------------ domain randomization
// dr_utils.generate_random_samples: the schedule scaling, then one draw of the descriptor's distribution
// (gaussian: np.random.normal(mu, var) = mu + var z).  Double precision like the reference's numpy.
__device__ double dr_sched(const mg_dr_desc& d, int64_t last_step) {
  if (d.schedule == MG_DR_SCHED_LINEAR)
    return 1.0 / (double)d.schedule_steps * (double)(last_step < d.schedule_steps ? last_step : d.schedule_steps);
  if (d.schedule == MG_DR_SCHED_CONSTANT) return last_step < d.schedule_steps ? 0.0 : 1.0;
  return 1.0;
}
__device__ double dr_sample(const mg_dr_desc& d, double sc, float u1, float u2) {
  double a = d.range[0], b = d.range[1];
  if (d.distribution == MG_DR_GAUSSIAN) {
    if (d.operation == MG_DR_ADDITIVE) { a *= sc; b *= sc; }
    else { b = b * sc; a = a * sc + 1.0 * (1.0 - sc); }
    const double z = sqrt(-2.0 * log(1.0 - (double)u1)) * cos(6.283185307179586 * (double)u2);
    return a + b * z;
  }
  if (d.operation == MG_DR_ADDITIVE) { a *= sc; b *= sc; }
  else { a = a * sc + 1.0 * (1.0 - sc); b = b * sc + 1.0 * (1.0 - sc); }
  if (d.distribution == MG_DR_LOGUNIFORM) return exp(log(a) + (log(b) - log(a)) * (double)u1);
  return a + (b - a) * (double)u1;
}
// dr_utils.get_bucketed_val: floor onto num_buckets buckets of the unscheduled range (uniform: [lo, hi];
// otherwise [mu - 2 sqrt(var), mu + 2 sqrt(var)]); below the first bucket Python's index -1 wraps to the last
__device__ double dr_bucket(const mg_dr_desc& d, double v) {
  double lo, hi;
  if (d.distribution == MG_DR_UNIFORM) { lo = d.range[0]; hi = d.range[1]; }
  else { lo = d.range[0] - 2.0 * sqrt((double)d.range[1]); hi = d.range[0] + 2.0 * sqrt((double)d.range[1]); }
  const int nb = d.num_buckets;
  int cnt = 0;  // bisect_right
  for (int i = 0; i < nb; i++)
    if ((hi - lo) * (double)i / (double)nb + lo <= v) cnt = i + 1;
  const int idx = cnt - 1 < 0 ? nb - 1 : cnt - 1;
  return (hi - lo) * (double)idx / (double)nb + lo;
}

// apply_randomizations' actor-property part for one actor per thread (vec_task.py:626-637, 746-842): the
// actor is randomized on the first call, or when randomize_buf >= frequency on a resetting step (then its
// counter restarts); each attribute element gets op(og, sample) (+ buckets) in its env_props column.
// Properties holding a setup_only attribute are only randomized on the first call.
__global__ __launch_bounds__(kBlock) void k_dr_apply(mg_dr_apply_args a) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= a.n) return;
  bool doit = a.first != 0;
  if (!doit) {
    int64_t rb = a.randomize_buf[e] + (a.increment ? 1 : 0);
    doit = rb >= (int64_t)a.frequency && a.reset_mask[e] != 0;
    if (doit) rb = 0;
    a.randomize_buf[e] = rb;
  }
  if (!doit) return;
  const uint64_t gid = (uint64_t)(a.env_offset + e);
  float* row = a.env_props + (size_t)a.stride * e;
  for (int i = 0; i < a.nattr; i++) {
    const mg_dr_attr at = a.attrs[i];
    const mg_dr_desc d = a.descs[at.desc];
    if (!a.first && !d.after_setup) continue;
    double smp;
    if (a.samples) {
      smp = (double)a.samples[(size_t)a.nattr * e + i];
    } else {
      const float u1 = mg::uniform01(a.seed, gid, a.counter, (uint32_t)(8192 + 2 * i));
      const float u2 = mg::uniform01(a.seed, gid, a.counter, (uint32_t)(8193 + 2 * i));
      smp = dr_sample(d, dr_sched(d, a.last_step), u1, u2);
    }
    double v = d.operation == MG_DR_SCALING ? (double)at.og * smp : (double)at.og + smp;
    if (d.num_buckets > 0) v = dr_bucket(d, v);
    row[at.slot] = (float)v;
  }
}

// noise_lambda (vec_task.py:684-720) over a flat tensor; corr is (re)drawn when refresh_corr is set
__global__ __launch_bounds__(kBlock) void k_dr_noise(mg_dr_noise_args a) {
#pragma clang fp contract(off)
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t gid = (uint64_t)(a.elem_offset + i);
    float c;
    if (a.refresh_corr) {
      if (a.injected_corr) {
        c = a.injected_corr[i];
      } else {
        const float u1 = mg::uniform01(a.seed, gid, a.counter, 4 * a.key), u2 = mg::uniform01(a.seed, gid, a.counter, 4 * a.key + 1);
        c = sqrtf(-2.0f * logf(1.0f - u1)) * cosf(6.28318530717958647f * u2);
      }
      a.corr[i] = c;
    } else {
      c = a.corr[i];
    }
    float z;
    if (a.injected) {
      z = a.injected[i];
    } else {
      const float u1 = mg::uniform01(a.seed, gid, a.counter, 4 * a.key + 2);
      if (a.distribution == MG_DR_GAUSSIAN) {
        const float u2 = mg::uniform01(a.seed, gid, a.counter, 4 * a.key + 3);
        z = sqrtf(-2.0f * logf(1.0f - u1)) * cosf(6.28318530717958647f * u2);
      } else {
        z = u1;
      }
    }
    const float cc = c * a.c_scale + a.c_shift;
    const float nz = (cc + z * a.scale) + a.shift;
    const float x = a.operation == MG_DR_SCALING ? a.x[i] * nz : a.x[i] + nz;
    a.x[i] = x;
    if (a.x_clamped) a.x_clamped[i] = fminf(fmaxf(x, -a.clip), a.clip);
  }
}

// ------------------------------------------------------------------------------------------------ C ABI
extern "C" {

const char* mg_last_error(void) { return g_err.c_str(); }
int mg_version(void) { return MG_VERSION; }
size_t mg_model_sizeof(void) { return sizeof(mg_model); }
size_t mg_task_params_sizeof(void) { return sizeof(mg_task_params); }
size_t mg_task_buffers_sizeof(void) { return sizeof(mg_task_buffers); }
size_t mg_sim_params_sizeof(void) { return sizeof(mg_sim_params); }
size_t mg_state_views_sizeof(void) { return sizeof(mg_state_views); }
size_t mg_dr_desc_sizeof(void) { return sizeof(mg_dr_desc); }
size_t mg_dr_apply_args_sizeof(void) { return sizeof(mg_dr_apply_args); }
size_t mg_dr_noise_args_sizeof(void) { return sizeof(mg_dr_noise_args); }

// Profiling aid: per-phase shader cycles summed over all waves (blocks < 65536) since the last reset (phase-timing
// build only; returns MG_EINVAL otherwise).  Phases: 0 FK, 1 ABA (+tendons), 2 collide (+object
// free step), 3 rows, 4 row Jacobians / W, 5 test solves, 6 PGS, 7 integrate, 8 outputs, 9 task layer +
// write-back, 13 constraint rows (count), 14 load + pre-physics, 15 substep entry.
#ifdef MG_PHASE_TIMING
static unsigned long long* g_phase_host_buf = nullptr;  // the per-wave rows (kPhaseCap x MG_NUM_PHASES)
#endif

int mg_debug_phase_cycles(uint64_t* out, int32_t reset) {
#ifdef MG_PHASE_TIMING
  constexpr int kPhaseCap = 1 << 16;  // blocks tracked (step_kernels.hpp)
  unsigned long long*& buf = g_phase_host_buf;
  const size_t bytes = (size_t)kPhaseCap * MG_NUM_PHASES * sizeof(unsigned long long);
  if (!buf) {  // first call: allocate + zero the per-wave rows and publish them to the kernels
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMemset(buf, 0, bytes) != hipSuccess)
      return fail(MG_EDEVICE, "mg_debug_phase_cycles: buffer setup failed");
    if (int rc = publish_all(buf, std::make_integer_sequence<int, MG_NUM_INST>{})) return rc;
    if (hipDeviceSynchronize() != hipSuccess) return fail(MG_EDEVICE, "mg_debug_phase_cycles: sync failed");
    if (out) memset(out, 0, MG_NUM_PHASES * sizeof(uint64_t));
    return MG_OK;
  }
  if (hipDeviceSynchronize() != hipSuccess) return fail(MG_EDEVICE, "mg_debug_phase_cycles: sync failed");
  if (out) {
    std::vector<unsigned long long> h((size_t)kPhaseCap * MG_NUM_PHASES);
    if (hipMemcpy(h.data(), buf, bytes, hipMemcpyDeviceToHost) != hipSuccess)
      return fail(MG_EDEVICE, "mg_debug_phase_cycles: copy failed");
    for (int i = 0; i < MG_NUM_PHASES; i++) out[i] = 0;
    for (size_t w = 0; w < (size_t)kPhaseCap; w++)
      for (int i = 0; i < MG_NUM_PHASES; i++) out[i] += h[MG_NUM_PHASES * w + i];
  }
  if (reset && hipMemset(buf, 0, bytes) != hipSuccess) return fail(MG_EDEVICE, "mg_debug_phase_cycles: reset failed");
  if (hipDeviceSynchronize() != hipSuccess) return fail(MG_EDEVICE, "mg_debug_phase_cycles: sync failed");
  return MG_OK;
#else
  (void)out;
  (void)reset;
  return fail(MG_EINVAL, "mg_debug_phase_cycles: library built without MG_PHASE_TIMING");
#endif
}

// Profiling aid: the per-item rows behind mg_debug_phase_cycles (an item = one wave's 64 / T teams; rows of
// MG_NUM_PHASES cycle counts, summed since the last reset), the first `cap` items.  Phase-timing build only.
int mg_debug_phase_waves(uint64_t* out, int32_t cap) {
#ifdef MG_PHASE_TIMING
  constexpr int kPhaseCap = 1 << 16;
  if (!out || cap < 0 || cap > kPhaseCap) return fail(MG_EINVAL, "mg_debug_phase_waves: bad arguments");
  if (!g_phase_host_buf) return fail(MG_EINVAL, "mg_debug_phase_waves: call mg_debug_phase_cycles first");
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemcpy(out, g_phase_host_buf, (size_t)cap * MG_NUM_PHASES * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess)
    return fail(MG_EDEVICE, "mg_debug_phase_waves: copy failed");
  return MG_OK;
#else
  (void)out;
  (void)cap;
  return fail(MG_EINVAL, "mg_debug_phase_waves: library built without MG_PHASE_TIMING");
#endif
}

int mg_sim_create(const mg_model* model, const mg_sim_params* params, int32_t num_envs, int32_t device,
                  mg_sim** out) {
  if (!model || !params || !out || num_envs <= 0) return fail(MG_EINVAL, "mg_sim_create: bad arguments");
  if (model->num_nodes < 1 || model->num_nodes > MG_MAX_NODES || model->num_geoms > MG_MAX_GEOMS ||
      model->num_pairs > MG_MAX_PAIRS || model->num_sensors > MG_MAX_SENSORS || model->num_bodies > MG_MAX_BODIES)
    return fail(MG_EINVAL, "mg_sim_create: model tables out of range");
  for (int i = 1; i < model->num_nodes; i++)
    if (model->parent[i] < 0 || model->parent[i] >= i)
      return fail(MG_EINVAL, "mg_sim_create: nodes must be topologically ordered (parent < child)");
  if (params->substeps < 1 || params->dt <= 0.0f || params->max_contacts < 0)
    return fail(MG_EINVAL, "mg_sim_create: bad sim params");
#ifdef MG_EXP_CLAMP_CONTACTS  // occupancy experiments only: the contact capacity clamped (never a shipped build)
  const_cast<mg_sim_params*>(params)->max_contacts =
      params->max_contacts < MG_EXP_CLAMP_CONTACTS ? params->max_contacts : MG_EXP_CLAMP_CONTACTS;
#endif
  if ((params->solver_type != MG_SOLVER_PGS && params->solver_type != MG_SOLVER_TGS) || params->vel_iters < 0)
    return fail(MG_EINVAL, "mg_sim_create: solver_type must be MG_SOLVER_PGS or MG_SOLVER_TGS, vel_iters >= 0");
  // the exact hull-object candidates are computed before the tree phases (team_physics.hpp hull_stage), from
  // the fixed root's pose: a convex-mesh geom colliding with a block / pen object must sit on that root
  if (model->obj_type == MG_GT_BOX || model->obj_type == MG_GT_CAPSULE)
    for (int g = 0; g < model->num_geoms; g++)
      if (model->geom_type[g] == MG_GT_CONVEX && (model->geom_filter[g] & MG_COLLIDE_OBJECT) &&
          (model->geom_node[g] != 0 || !model->fixed_base))
        return fail(MG_EINVAL, "mg_sim_create: a convex-mesh geom against the object must be on the fixed root");
  {  // one convex-mesh geom may collide with the object: the LDS tile stages one hull (build_tile's hullg)
    int ncvx = 0;
    for (int g = 0; g < model->num_geoms; g++)
      ncvx += model->geom_type[g] == MG_GT_CONVEX && (model->geom_filter[g] & MG_COLLIDE_OBJECT);
    if (model->obj_type && ncvx > 1)
      return fail(MG_EINVAL, "mg_sim_create: at most one convex-mesh geom may collide with the object");
  }
  if (hipSetDevice(device) != hipSuccess) return fail(MG_EDEVICE, "mg_sim_create: hipSetDevice failed");
  mg_sim* s = new (std::nothrow) mg_sim();
  if (!s) return fail(MG_ENOMEM, "mg_sim_create: out of host memory");
  s->host_model = *model;
  s->params = *params;
  s->n = num_envs;
  s->device = device;
  s->bound = false;
  if (hipMalloc(&s->d_model, sizeof(mg_model)) != hipSuccess) {
    delete s;
    return fail(MG_ENOMEM, "mg_sim_create: hipMalloc(model) failed");
  }
  if (hipMemcpy(s->d_model, model, sizeof(mg_model), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(s->d_model);
    delete s;
    return fail(MG_EDEVICE, "mg_sim_create: model upload failed");
  }
  // the LDS model tile of the instance that will run this model, prebuilt once on the host; a model no
  // instance fits is still created (its launches report MG_ECAPACITY)
  s->d_tile = nullptr;
  // work ordering (MgOrder, step_kernels.hpp: the envs in descending order of their last row counts)
  s->order_mode = kOrderOff;
  s->order_steps = 0;
  s->sort_every = 1;
  s->order_valid = false;
  s->d_bq = nullptr;
  s->d_blist = nullptr;
  s->bq_cap = 0;
  s->order_unit = s->order_agents = 1;
  s->d_order = nullptr;
  s->d_cost = nullptr;
  s->d_osort = nullptr;
  s->d_span = nullptr;
  s->span_cap = s->span_next = s->span_stride = 0;
  // default (same box, M env-steps/s unordered -> ordered): the sort for ShadowHand and Humanoid from
  // 16,384 envs and for Ant from 32,768 one-agent envs (ShadowHand 16,384 18.9 -> 20.1, in-kernel lists 20.0;
  // Humanoid 32,768 33.9 -> 37.3, lists 37.0; Ant 65,536 152.7 -> 157.8, lists 119.4: their hot-bucket atomics);
  // off for MA-Ant (8,192 -0.8 %, 65,536 -1.0 % sorted), Cartpole and the smaller batches (Ant 16,384 within
  // noise, ShadowHand 4,096 -2 %: the sort's two launches outweigh the tail they save).
  // MIGYM_ORDER = off | lists | sort | sort:K (sort every K-th launch only; A/B: the order goes stale within two
  // steps) overrides.
  {
    const int T = mgi::team_size(s->host_model, s->params.max_contacts);
    const int A = params->agents > 1 ? params->agents : 1;
    if (T >= 32) s->order_mode = num_envs >= 16384 ? kOrderSort : kOrderOff;
    else if (T == 16 && A == 1) s->order_mode = num_envs >= 32768 ? kOrderSort : kOrderOff;
  }
  s->lds_pad = 0;
  if (const char* e = getenv("MIGYM_LDS_PAD")) s->lds_pad = atoi(e) > 0 ? atoi(e) : 0;
  // team LDS layout: by default the classic layout for a batch the classic kernel holds resident
  // (dispatch.hpp kCompactMinWaves) and the compact 12-wave layout above it.  The two layouts round differently, so
  // a shard is the bit-identical slice of a bigger rollout only when both pick the same layout:
  // MIGYM_LAYOUT = compact | classic pins it (auto: the default).
  s->layout_n = s->n;
  if (const char* e = getenv("MIGYM_LAYOUT")) {
    if (!strcmp(e, "classic")) s->layout_n = 0;
    else if (!strcmp(e, "compact")) s->layout_n = 1L << 40;
    else if (strcmp(e, "auto")) {
      mg_sim_destroy(s);
      return fail(MG_EINVAL, "mg_sim_create: MIGYM_LAYOUT must be auto, compact or classic");
    }
  }
  if (const char* e = getenv("MIGYM_ORDER")) {
    if (!strcmp(e, "off")) s->order_mode = kOrderOff;
    else if (!strcmp(e, "lists")) s->order_mode = kOrderLists;
    else if (!strcmp(e, "sort")) s->order_mode = kOrderSort;
    else if (!strncmp(e, "sort:", 5) && atoi(e + 5) > 0) {
      s->order_mode = kOrderSort;
      s->sort_every = atoi(e + 5);
    } else {
      mg_sim_destroy(s);
      return fail(MG_EINVAL, "mg_sim_create: MIGYM_ORDER must be off, lists, sort or sort:K (K > 0)");
    }
  }
  if (s->order_mode != kOrderOff) {
    const int A = params->agents > 1 ? params->agents : 1;
    s->order_agents = A;
    s->order_unit = A;
    if (MG_SORT_WAVE_UNITS && s->order_mode == kOrderSort && A == 1 && s->host_model.obj_type == 0) {
      const int T = mgi::team_size(s->host_model, s->params.max_contacts), U = T > 0 ? 64 / T : 1;
      if (U > 1 && num_envs % U == 0) s->order_unit = U;  // (a ragged batch keeps one env per unit)
    }
    s->bq_cap = (num_envs + s->order_unit - 1) / s->order_unit;
    const size_t nu = (size_t)s->bq_cap, nb = (nu + 255) / 256;
    const bool ok = s->order_mode == kOrderLists
        ? hipMalloc(&s->d_bq, sizeof(unsigned) * (2 * kOrderBuckets + 1)) == hipSuccess &&
              hipMemset(s->d_bq, 0, sizeof(unsigned) * (2 * kOrderBuckets + 1)) == hipSuccess &&
              hipMalloc(&s->d_blist, sizeof(int) * 2 * (size_t)kOrderBuckets * nu) == hipSuccess
        : hipMalloc(&s->d_osort, sizeof(unsigned) * (kSortTot + 256 * nb) + sizeof(unsigned short) * (nu + 2)) == hipSuccess &&
              hipMemset(s->d_osort, 0, sizeof(unsigned) * kSortTot) == hipSuccess &&
              hipMalloc(&s->d_order, sizeof(int) * nu) == hipSuccess &&
              hipMalloc(&s->d_cost, nu) == hipSuccess && hipMemset(s->d_cost, 0, nu) == hipSuccess;
    if (!ok) {
      mg_sim_destroy(s);
      return fail(MG_ENOMEM, "mg_sim_create: hipMalloc(work order) failed");
    }
  }
  // the step kernels' work-queue counters: zero here, and zeroed again by the last wave of every launch
  if (hipMalloc(&s->d_wq, 2 * sizeof(unsigned)) != hipSuccess || hipMemset(s->d_wq, 0, 2 * sizeof(unsigned)) != hipSuccess) {
    mg_sim_destroy(s);
    return fail(MG_ENOMEM, "mg_sim_create: hipMalloc(work queue) failed");
  }
  if (mgi::team_size(s->host_model, s->params.max_contacts) > 0) {
    const int rc = mgi::dispatch<mgi::BuildTile>(s->host_model, s->params.max_contacts, s->layout_n, s);
    if (rc) {
      mg_sim_destroy(s);
      return rc;
    }
  }
  *out = s;
  return MG_OK;
}

int mg_sim_bind(mg_sim* sim, const mg_state_views* views) {
  if (!sim || !views || !views->root_states || !views->dof_state) return fail(MG_EINVAL, "mg_sim_bind: bad views");
  if (sim->host_model.num_sensors > 0 && !views->sensors)
    return fail(MG_EINVAL, "mg_sim_bind: model has force sensors but no sensor buffer");
  if (views->env_props && views->env_props_stride < mg_env_props_layout(&sim->host_model, nullptr))
    return fail(MG_EINVAL, "mg_sim_bind: env_props_stride is shorter than mg_env_props_layout's row");
  sim->views = *views;
  sim->bound = true;
  return MG_OK;
}

int mg_sim_simulate(mg_sim* sim, void* stream) {
  if (!sim || !sim->bound) return fail(MG_EINVAL, "mg_sim_simulate: sim not bound");
  int rc = mgi::dispatch<mgi::RunSimulate>(sim->host_model, sim->params.max_contacts, sim->layout_n, (hipStream_t)stream,
                                 (const mg_sim*)sim);
  if (rc) return rc;
  return check_launch("mg_sim_simulate");
}

int mg_sim_set_params(mg_sim* sim, const mg_sim_params* params) {
  if (!sim || !params || params->substeps < 1 || params->dt <= 0.0f || params->max_contacts < 0)
    return fail(MG_EINVAL, "mg_sim_set_params: bad arguments");
  if (params->max_contacts != sim->params.max_contacts || params->agents != sim->params.agents)
    return fail(MG_EINVAL, "mg_sim_set_params: max_contacts / agents are fixed at mg_sim_create");
  if ((params->solver_type != MG_SOLVER_PGS && params->solver_type != MG_SOLVER_TGS) || params->vel_iters < 0)
    return fail(MG_EINVAL, "mg_sim_set_params: solver_type must be MG_SOLVER_PGS or MG_SOLVER_TGS, vel_iters >= 0");
  sim->params = *params;  // taken by value by every later launch
  return MG_OK;
}

int mg_env_props_layout(const mg_model* m, int32_t offsets[4]) {
  if (!m) return fail(MG_EINVAL, "mg_env_props_layout: bad model");
  const int o0 = 0, o1 = MG_EP_NODE_WIDTH * m->num_nodes, o2 = o1 + m->num_geoms, o3 = o2 + 2 * m->num_tendons;
  if (offsets) { offsets[0] = o0; offsets[1] = o1; offsets[2] = o2; offsets[3] = o3; }
  return (o3 + 4 + 3) & ~3;
}

int mg_env_props_defaults(const mg_model* m, float* row) {
  if (!m || !row) return fail(MG_EINVAL, "mg_env_props_defaults: bad arguments");
  int32_t off[4];
  const int stride = mg_env_props_layout(m, off);
  for (int k = 0; k < stride; k++) row[k] = 0.0f;
  for (int i = 0; i < m->num_nodes; i++) {
    float* r = row + off[MG_EP_NODE] + MG_EP_NODE_WIDTH * i;
    r[0] = m->mass[i]; r[1] = m->armature[i]; r[2] = m->damping[i]; r[3] = m->stiffness[i];
    r[4] = m->lower[i]; r[5] = m->upper[i]; r[6] = m->drive_kp[i]; r[7] = m->effort_limit[i];
    r[8] = m->frictionloss[i];
  }
  for (int g = 0; g < m->num_geoms; g++) row[off[MG_EP_GEOM] + g] = 1.0f;  // shape friction (build-defined default)
  for (int q = 0; q < m->num_tendons; q++) {
    row[off[MG_EP_TENDON] + 2 * q] = m->tendon_limit_stiffness[q];
    row[off[MG_EP_TENDON] + 2 * q + 1] = m->tendon_damping[q];
  }
  float* o = row + off[MG_EP_OBJECT];
  o[0] = m->obj_mass; o[1] = 1.0f; o[2] = 1.0f; o[3] = 0.0f;
  return MG_OK;
}

int mg_dr_apply(const mg_dr_apply_args* a, void* stream) {
  if (!a || a->n < 0 || a->nattr < 0 || (a->nattr > 0 && (!a->descs || !a->attrs)) || !a->env_props ||
      a->stride <= 0 || (!a->first && (!a->reset_mask || !a->randomize_buf)))
    return fail(MG_EINVAL, "mg_dr_apply: bad arguments");
  if (a->n == 0) return MG_OK;
  hipLaunchKernelGGL(k_dr_apply, dim3(grid_for(a->n)), dim3(kBlock), 0, (hipStream_t)stream, *a);
  return check_launch("mg_dr_apply");
}

int mg_dr_noise(const mg_dr_noise_args* a, void* stream) {
  if (!a || !a->x || !a->corr || a->n < 0) return fail(MG_EINVAL, "mg_dr_noise: bad arguments");
  if (a->n == 0) return MG_OK;
  const int64_t blocks = (a->n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(k_dr_noise, dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(kBlock), 0,
                     (hipStream_t)stream, *a);
  return check_launch("mg_dr_noise");
}

int mg_sim_destroy(mg_sim* sim) {
  if (!sim) return MG_OK;
  if (sim->d_model) (void)hipFree(sim->d_model);
  if (sim->d_tile) (void)hipFree(sim->d_tile);
  if (sim->d_wq) (void)hipFree(sim->d_wq);
  if (sim->d_bq) (void)hipFree(sim->d_bq);
  if (sim->d_blist) (void)hipFree(sim->d_blist);
  if (sim->d_order) (void)hipFree(sim->d_order);
  if (sim->d_cost) (void)hipFree(sim->d_cost);
  if (sim->d_osort) (void)hipFree(sim->d_osort);
  if (sim->d_span) (void)hipFree(sim->d_span);
  delete sim;
  return MG_OK;
}

int mg_kernel_span_begin(mg_sim* sim, int32_t cap) {
  if (!sim || cap < 0 || cap > (int32_t)(sizeof(sim->span_waves) / sizeof(sim->span_waves[0])))
    return fail(MG_EINVAL, "mg_kernel_span_begin: bad arguments (cap 0..1024)");
  if (sim->d_span) (void)hipFree(sim->d_span);
  sim->d_span = nullptr;
  sim->span_cap = sim->span_next = 0;
  if (cap == 0) return MG_OK;
  // a launch's waves: one per 64 / T actors (T = the instance's team size), rounded up to whole blocks (<= 8 waves)
  const int T = mgi::team_size(sim->host_model, sim->params.max_contacts);
  sim->span_stride = (int)(((int64_t)sim->n * (T > 0 ? T : 64) + 63) / 64) + 8;
  const size_t bytes = sizeof(unsigned long long) * 2 * (size_t)sim->span_stride * (size_t)cap;
  if (hipMalloc(&sim->d_span, bytes) != hipSuccess) {
    sim->d_span = nullptr;
    return fail(MG_ENOMEM, "mg_kernel_span_begin: hipMalloc failed");
  }
  // zeros: a launch that records nothing (a build without the hooks) reads back as a zero span
  if (hipMemset(sim->d_span, 0, bytes) != hipSuccess) return fail(MG_EDEVICE, "mg_kernel_span_begin: memset failed");
  sim->span_cap = cap;
  return MG_OK;
}

int mg_kernel_span_read(mg_sim* sim, double* ms, int32_t cap, int32_t* n_out) {
  if (!sim || !ms || !n_out || cap < 0) return fail(MG_EINVAL, "mg_kernel_span_read: bad arguments");
  *n_out = 0;
  const int n = sim->span_next < cap ? sim->span_next : cap;
  if (!sim->d_span || n == 0) return MG_OK;
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, sim->device) != hipSuccess || khz <= 0)
    return fail(MG_EDEVICE, "mg_kernel_span_read: wall clock rate query failed");
  if (hipDeviceSynchronize() != hipSuccess) return fail(MG_EDEVICE, "mg_kernel_span_read: sync failed");
  std::vector<unsigned long long> h;
  for (int i = 0; i < n; i++) {
    const int w = sim->span_waves[i];
    h.resize(2 * (size_t)w);
    if (hipMemcpy(h.data(), sim->d_span + 2 * (size_t)sim->span_stride * i, h.size() * sizeof(unsigned long long),
                  hipMemcpyDeviceToHost) != hipSuccess)
      return fail(MG_EDEVICE, "mg_kernel_span_read: copy failed");
    unsigned long long t0 = ~0ull, t1 = 0;
    for (int k = 0; k < w; k++) {
      t0 = h[2 * k] < t0 ? h[2 * k] : t0;
      t1 = h[2 * k + 1] > t1 ? h[2 * k + 1] : t1;
    }
    ms[i] = t1 >= t0 ? (double)(t1 - t0) / (double)khz : -1.0;
  }
  *n_out = n;
  return MG_OK;
}

int mg_kernel_span_waves(mg_sim* sim, int32_t launch, uint64_t* out, int32_t cap, int32_t* n_out) {
  if (!sim || !out || !n_out || cap < 0 || launch < 0) return fail(MG_EINVAL, "mg_kernel_span_waves: bad arguments");
  *n_out = 0;
  if (!sim->d_span || launch >= sim->span_next) return MG_OK;
  const int w = sim->span_waves[launch] < cap ? sim->span_waves[launch] : cap;
  if (hipDeviceSynchronize() != hipSuccess) return fail(MG_EDEVICE, "mg_kernel_span_waves: sync failed");
  if (w > 0 && hipMemcpy(out, sim->d_span + 2 * (size_t)sim->span_stride * launch, 2 * (size_t)w * sizeof(uint64_t),
                         hipMemcpyDeviceToHost) != hipSuccess)
    return fail(MG_EDEVICE, "mg_kernel_span_waves: copy failed");
  *n_out = w;
  return MG_OK;
}

int mg_work_order(mg_sim* sim, int32_t* order, uint8_t* cost, int32_t cap, int32_t* mode, int32_t* n_out) {
  if (!sim || !mode || !n_out || cap < 0) return fail(MG_EINVAL, "mg_work_order: bad arguments");
  *mode = sim->order_mode;
  *n_out = 0;
  if (sim->order_mode != kOrderSort) return MG_OK;
  const int n = sim->bq_cap < cap ? sim->bq_cap : cap;
  if (hipDeviceSynchronize() != hipSuccess) return fail(MG_EDEVICE, "mg_work_order: sync failed");
  if (order) {
    if (sim->order_valid && sim->order_steps > 1) {
      if (n > 0 && hipMemcpy(order, sim->d_order, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess)
        return fail(MG_EDEVICE, "mg_work_order: copy failed");
    } else {
      for (int i = 0; i < n; i++) order[i] = i;  // no sort has run yet: the launches took the slots in order
    }
  }
  if (cost && n > 0 && hipMemcpy(cost, sim->d_cost, (size_t)n, hipMemcpyDeviceToHost) != hipSuccess)
    return fail(MG_EDEVICE, "mg_work_order: copy failed");
  *n_out = n;
  return MG_OK;
}

int mg_sim_kernel_layout(mg_sim* sim, int32_t* team_lanes, int32_t* compact) {
  if (!sim || !team_lanes || !compact) return fail(MG_EINVAL, "mg_sim_kernel_layout: bad arguments");
  *team_lanes = 0;
  *compact = 0;
  if (mgi::team_size(sim->host_model, sim->params.max_contacts) <= 0) return MG_OK;  // no instance fits: no team kernel
  return mgi::dispatch<mgi::InstanceOf>(sim->host_model, sim->params.max_contacts, sim->layout_n, team_lanes, compact);
}

int mg_set_indexed(mg_sim* sim, int32_t which, const float* src, const int32_t* idx, int32_t n, void* stream) {
  if (!sim || !sim->bound || !src || (n > 0 && !idx)) return fail(MG_EINVAL, "mg_set_indexed: bad arguments");
  if (n == 0) return MG_OK;
  float* dst;
  int row;
  if (which == MG_SET_ROOT_STATE) {
    dst = sim->views.root_states;
    row = 13;
  } else if (which == MG_SET_DOF_STATE) {
    dst = sim->views.dof_state;
    row = 2 * sim->host_model.num_dofs;
  } else if (which == MG_SET_DOF_TARGET) {
    dst = const_cast<float*>(sim->views.dof_targets);
    row = sim->host_model.num_dofs;
    if (!dst) return fail(MG_EINVAL, "mg_set_indexed: no dof_targets bound");
  } else {
    return fail(MG_EINVAL, "mg_set_indexed: unknown target");
  }
  if (dst == src) return MG_OK;  // caller wrote into the bound buffer itself (gym views alias sim memory)
  const int total = n * row;
  // hand-task envs: actor ids are global (3 per env: hand, object, goal); DOF rows belong to the hand
  const int div = (which != MG_SET_ROOT_STATE && sim->host_model.obj_type) ? 3 : 1;
  hipLaunchKernelGGL(k_set_indexed, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream, dst, src, idx, n,
                     row, div);
  return check_launch("mg_set_indexed");
}

int mg_compute_observations(const mg_task_params* tp, int32_t n, const float* root_states, const float* dof_state,
                            const float* dof_force, const float* sensors, const float* actions, float* potentials,
                            float* prev_potentials, float* up_vec, float* heading_vec, float* obs, void* stream) {
  if (!tp || n < 0 || !dof_state || !obs || !actions) return fail(MG_EINVAL, "mg_compute_observations: bad args");
  if (tp->task_id != MG_TASK_CARTPOLE && (!root_states || !potentials || !prev_potentials || !up_vec || !heading_vec))
    return fail(MG_EINVAL, "mg_compute_observations: locomotion task needs root/potential buffers");
  if (n == 0) return MG_OK;
  hipLaunchKernelGGL(k_observations, dim3(grid_for(n)), dim3(kBlock), 0, (hipStream_t)stream, *tp, n, root_states,
                     dof_state, dof_force, sensors, actions, potentials, prev_potentials, up_vec, heading_vec, obs);
  return check_launch("mg_compute_observations");
}

int mg_compute_reward(const mg_task_params* tp, int32_t n, const float* obs, const float* actions,
                      const float* potentials, const float* prev_potentials, const int64_t* progress, int64_t* reset,
                      float* rew, void* stream) {
  if (!tp || n < 0 || !obs || !actions || !progress || !reset || !rew) return fail(MG_EINVAL, "mg_compute_reward");
  if (tp->task_id != MG_TASK_CARTPOLE && (!potentials || !prev_potentials))
    return fail(MG_EINVAL, "mg_compute_reward: locomotion task needs potentials");
  if (n == 0) return MG_OK;
  hipLaunchKernelGGL(k_reward, dim3(grid_for(n)), dim3(kBlock), 0, (hipStream_t)stream, *tp, n, obs, actions,
                     potentials, prev_potentials, progress, reset, rew);
  return check_launch("mg_compute_reward");
}

static int hand_args_ok(const mg_task_params* tp, const mg_state_views& v, const mg_task_buffers* tb,
                        const char* who) {
  if (!v.dof_targets || !v.rigid_body_states || !v.sensors || !v.dof_force || !tb->prev_targets ||
      !tb->goal_states || !tb->reset_goal || !tb->successes || !tb->consecutive_successes ||
      !tb->reduce_scratch || !tb->actions_out)
    return fail(MG_EINVAL, std::string(who) + ": ShadowHand needs dof_targets, rigid_body_states, sensors, "
                                              "dof_force and the hand task buffers");
  if (tp->num_dofs <= 0 || tp->num_dofs > MG_MAX_HAND_DOFS || tp->num_actions > MG_MAX_HAND_DOFS)
    return fail(MG_EINVAL, std::string(who) + ": bad hand DOF / action count");
  // obs_map / state_map hold 256 columns; the fused kernel's LDS row holds 212 (checked at launch)
  if (tp->num_obs <= 0 || tp->num_obs > 256 || tp->num_states < 0 || tp->num_states > 256)
    return fail(MG_EINVAL, std::string(who) + ": bad hand observation / state count");
  return MG_OK;
}

int mg_pre_physics(mg_sim* sim, const mg_task_params* tp, const mg_state_views* views, const mg_task_buffers* tb,
                   int32_t n, void* stream) {
  if (!tp || !tb || !tb->actions) return fail(MG_EINVAL, "mg_pre_physics: bad args");
  mg_state_views v;
  int nd;
  if (sim) {
    if (!sim->bound) return fail(MG_EINVAL, "mg_pre_physics: sim not bound");
    v = sim->views;
    n = sim->n;
    nd = sim->host_model.num_dofs;
  } else {
    if (!views) return fail(MG_EINVAL, "mg_pre_physics: need views without a sim");
    v = *views;
    nd = tp->task_id == MG_TASK_SHADOW_HAND ? tp->num_dofs : (tp->task_id == MG_TASK_CARTPOLE ? 2 : tp->num_actions);
  }
  if (n == 0) return MG_OK;
  if (tp->task_id == MG_TASK_SHADOW_HAND) {
    int rc = hand_args_ok(tp, v, tb, "mg_pre_physics");
    if (rc) return rc;
    hipLaunchKernelGGL(k_hand_pre, dim3(grid_for(n)), dim3(kBlock), 0, (hipStream_t)stream, *tp, v, *tb, n, nd);
  } else {
    if (!v.dof_actuation) return fail(MG_EINVAL, "mg_pre_physics: locomotion task needs dof_actuation");
    hipLaunchKernelGGL(k_pre_loco, dim3(grid_for(n * nd)), dim3(kBlock), 0, (hipStream_t)stream, *tp, v, *tb, n,
                       nd);
  }
  return check_launch("mg_pre_physics");
}

int mg_post_physics(mg_sim* sim, const mg_task_params* tp, const mg_state_views* views, const mg_task_buffers* tb,
                    int32_t n, void* stream) {
  if (!tp || !tb) return fail(MG_EINVAL, "mg_post_physics: bad args");
  if (tp->num_actions > 64) return fail(MG_EINVAL, "mg_post_physics: num_actions > 64");
  if (tp->num_agents > 1 && (64 % tp->num_agents != 0 || tp->num_agents > MG_MAX_AGENTS ||
                             (sim ? sim->n : n) % tp->num_agents != 0))
    return fail(MG_EINVAL, "mg_post_physics: num_agents must divide 64 and the actor count");
  mg_state_views v;
  if (sim) {
    if (!sim->bound) return fail(MG_EINVAL, "mg_post_physics: sim not bound");
    v = sim->views;
    n = sim->n;
  } else {
    if (!views) return fail(MG_EINVAL, "mg_post_physics: need views without a sim");
    v = *views;
  }
  if (n == 0) return MG_OK;
  if (tp->task_id == MG_TASK_SHADOW_HAND) {
    int rc = hand_args_ok(tp, v, tb, "mg_post_physics");
    if (rc) return rc;
    hipLaunchKernelGGL(k_hand_post, dim3(grid_for(n)), dim3(kBlock), 0, (hipStream_t)stream, *tp, v, *tb, n,
                       tp->num_dofs);
    if (!tb->defer_finalize)
      hipLaunchKernelGGL(k_hand_finalize, dim3(1), dim3(64), 0, (hipStream_t)stream, *tp, *tb);
    return check_launch("mg_post_physics");
  }
  hipLaunchKernelGGL(k_post_physics, dim3(grid_for(n)), dim3(kBlock), 0, (hipStream_t)stream, *tp, v, *tb, n);
  return check_launch("mg_post_physics");
}

// Work ordering, sort mode (kOrderSort): a counting sort of the env units by the last launch's row counts,
// descending (the largest first), in two grid-wide passes of 256-unit blocks.  Pass 1 (k_ohist): each block's
// histogram in LDS -- the lanes of one key aggregated into one LDS add per key and wave, since a few hot bins would
// otherwise serialise every add -- then one global atomic per block and used bin reserves the block's range inside
// the bin, and each unit keeps its rank inside its block's range.  Pass 2 (k_oscatter): the bins' starts (a block
// scan of the 256 totals) and each unit's slot.  Where a unit lands inside its bin never changes a result, only
// which units share a wave.  The step kernel that runs this permutation zeroes the totals for the next sort
// (MgOrder::tot_clear), so the launches carry no host-side state and a captured graph replays them any number of times.
// (Fusing the histogram into the step kernel -- a global add per env -- and placing by per-bin cursors measured far
// slower: one hot bin's atomics serialise, Ant 65,536 156.0 -> 108.5 M)
__global__ __launch_bounds__(256) void k_ohist(const unsigned char* __restrict__ cost, int nu,
                                               unsigned* __restrict__ tot, unsigned* __restrict__ bbase,
                                               unsigned short* __restrict__ rank) {
  __shared__ unsigned h[256];
  h[threadIdx.x] = 0u;
  __syncthreads();
  const int u = (int)blockIdx.x * 256 + (int)threadIdx.x;
  const int lane = (int)(threadIdx.x & 63);
  const int key = u < nu ? 255 - (int)cost[u] : -1;
  unsigned r = 0u;
  unsigned long long rem = __ballot(key >= 0);
  while (rem) {
    const int leader = __builtin_ctzll(rem);
    const int k = __shfl(key, leader);
    const unsigned long long same = __ballot(key == k) & rem;
    unsigned base = 0u;
    if (lane == leader) base = atomicAdd(&h[k], (unsigned)__popcll(same));
    base = (unsigned)__shfl((int)base, leader);
    if ((same >> lane) & 1ull) r = base + (unsigned)__popcll(same & ((1ull << lane) - 1ull));
    rem &= ~same;
  }
  __syncthreads();
  const unsigned c = h[threadIdx.x];
  bbase[(size_t)blockIdx.x * 256 + threadIdx.x] = c ? atomicAdd(&tot[256 * (blockIdx.x % kSortRep) + threadIdx.x], c) : 0u;
  if (u < nu) rank[u] = (unsigned short)r;
}
__global__ __launch_bounds__(256) void k_oscatter(const unsigned char* __restrict__ cost, int nu,
                                                  const unsigned* __restrict__ tot, const unsigned* __restrict__ bbase,
                                                  const unsigned short* __restrict__ rank, int* __restrict__ order) {
  __shared__ unsigned wsum[4], start[256];
  const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
  // the bin's total over the copies, and this block's copy's offset inside the bin (the copies before it)
  const int rep = (int)(blockIdx.x % kSortRep);
  unsigned v = 0u, roff = 0u;
#pragma unroll
  for (int k = 0; k < kSortRep; k++) {
    const unsigned x = tot[256 * k + threadIdx.x];
    roff += k < rep ? x : 0u;
    v += x;
  }
  unsigned inc = v;
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned y = (unsigned)__shfl_up((int)inc, d);
    inc += lane >= d ? y : 0u;
  }
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  unsigned off = 0u;
  for (int w = 0; w < wv; w++) off += wsum[w];
  start[threadIdx.x] = off + inc - v + roff;
  __syncthreads();
  const int u = (int)blockIdx.x * 256 + (int)threadIdx.x;
  if (u < nu) {
    const int key = 255 - (int)cost[u];
    const unsigned pos = start[key] + bbase[(size_t)blockIdx.x * 256 + key] + rank[u];
    if (pos < (unsigned)nu) order[pos] = u;  // always, unless the totals were not cleared
  }
}

static int env_step(mg_sim* sim, const mg_task_params* tp, const mg_task_buffers* tb, const mg_replay* rp,
                    void* stream) {
  if (!sim || !sim->bound || !tp || !tb || !tb->actions || !tb->obs || !tb->rew || !tb->reset || !tb->progress ||
      !tb->timeout)
    return fail(MG_EINVAL, "mg_env_step: bad arguments");
  const bool hand = tp->task_id == MG_TASK_SHADOW_HAND;
  if (hand != (sim->host_model.obj_type != 0))
    return fail(MG_EINVAL, "mg_env_step: ShadowHand needs a model with a free object (and only it does)");
  if (hand) {
    int rc = hand_args_ok(tp, sim->views, tb, "mg_env_step");
    if (rc) return rc;
    if (tp->num_dofs != sim->host_model.num_dofs || tp->rb_per_env != sim->host_model.num_bodies + 2)
      return fail(MG_EINVAL, "mg_env_step: task DOF / rigid-body counts do not match the model");
  } else {
    if (tp->task_id != MG_TASK_CARTPOLE && (!tb->potentials || !tb->prev_potentials || !tb->up_vec || !tb->heading_vec))
      return fail(MG_EINVAL, "mg_env_step: locomotion task needs potential/up/heading buffers");
    if (tp->num_actions > sim->host_model.num_nodes && tp->task_id != MG_TASK_CARTPOLE)
      return fail(MG_EINVAL, "mg_env_step: more actions than DOFs");
    if (tp->num_actions > mgi::team_size(sim->host_model, sim->params.max_contacts))
      return fail(MG_EINVAL, "mg_env_step: more actions than lanes per actor");
  }
  if (tp->num_agents > 1) {
    // the agents of an env must be teams of one wave (ballot/shuffle exchange): A | 64/T
    const int T = mgi::team_size(sim->host_model, sim->params.max_contacts);
    if (T == 0 || tp->num_agents > MG_MAX_AGENTS || (64 / T) % tp->num_agents != 0 ||
        sim->n % tp->num_agents != 0)
      return fail(MG_EINVAL, "mg_env_step: num_agents must divide the envs per wave (64 / team size) "
                             "and the actor count");
  }
  if (tp->num_actions > 64 || tp->num_obs > 256 || tp->num_states > 256)
    return fail(MG_EINVAL, "mg_env_step: num_actions > 64, num_obs > 256 or num_states > 256");
  if (sim->order_mode == kOrderLists && !rp) {
    // the in-kernel lists alternate between two sets by the host's launch parity, which a captured graph would freeze
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing((hipStream_t)stream, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
      return fail(MG_EINVAL, "mg_env_step: MIGYM_ORDER=lists cannot be captured into a graph (use sort or off)");
  }
  if (sim->order_mode != kOrderOff && !rp) {
    const int A = tp->num_agents > 1 ? tp->num_agents : 1;
    if (A != sim->order_agents) return fail(MG_EINVAL, "mg_env_step: num_agents differs from mg_sim_params.agents");
    // the last launch's row counts -> this one's order (every sort_every-th ordered launch from the second on)
    if (sim->order_mode == kOrderSort && sim->order_valid && (sim->order_steps - 1) % sim->sort_every == 0) {
      const int nu = sim->bq_cap, nb = (nu + 255) / 256;
      unsigned* bbase = sim->d_osort + kSortTot;
      unsigned short* rank = reinterpret_cast<unsigned short*>(sim->d_osort + kSortTot + 256 * (size_t)nb);
      unsigned* tot = sim->d_osort;
      hipLaunchKernelGGL(k_ohist, dim3(nb), dim3(256), 0, (hipStream_t)stream, sim->d_cost, nu, tot, bbase, rank);
      hipLaunchKernelGGL(k_oscatter, dim3(nb), dim3(256), 0, (hipStream_t)stream, sim->d_cost, nu, tot, bbase, rank,
                         sim->d_order);
    }
  }
  int rc = mgi::dispatch<mgi::RunEnvStep>(sim->host_model, sim->params.max_contacts, sim->layout_n, (hipStream_t)stream,
                                          (const mg_sim*)sim, tp, tb, rp);
  if (rc) return rc;
  if (sim->order_mode != kOrderOff && !rp) {  // the launch wrote the next one's lists / row counts
    sim->order_steps++;
    sim->order_valid = true;
  }
  if (hand && !tb->defer_finalize)  // consecutive_successes running mean from the step's partial sums
    hipLaunchKernelGGL(k_hand_finalize, dim3(1), dim3(64), 0, (hipStream_t)stream, *tp, *tb);
  return check_launch(rp ? "mg_env_step_replay" : "mg_env_step");
}

int mg_env_step(mg_sim* sim, const mg_task_params* tp, const mg_task_buffers* tb, void* stream) {
  return env_step(sim, tp, tb, nullptr, stream);
}

int mg_reset_idx(mg_sim* sim, const mg_task_params* tp, const mg_task_buffers* tb, const int32_t* ids, int32_t n,
                 void* stream) {
  if (!sim || !sim->bound || !tp || !tb || n < 0 || (n > 0 && !ids) || !tb->reset || !tb->progress)
    return fail(MG_EINVAL, "mg_reset_idx: bad arguments");
  if (n == 0) return MG_OK;
  const bool hand = tp->task_id == MG_TASK_SHADOW_HAND;
  if (hand) {
    int rc = hand_args_ok(tp, sim->views, tb, "mg_reset_idx");
    if (rc) return rc;
  } else if (tp->task_id != MG_TASK_CARTPOLE && (!tb->potentials || !tb->prev_potentials)) {
    return fail(MG_EINVAL, "mg_reset_idx: locomotion task needs potential buffers");
  }
  if (tp->num_agents > MG_MAX_AGENTS) return fail(MG_EINVAL, "mg_reset_idx: num_agents > MG_MAX_AGENTS");
  mg_task_buffers t = *tb;
  t.step_counter = tb->step_counter | (1ull << 62);  // the manual-reset stream of the counter RNG
  hipLaunchKernelGGL(k_reset_idx, dim3(grid_for(n)), dim3(kBlock), 0, (hipStream_t)stream, *tp, sim->views, t, ids,
                     n, sim->n);
  return check_launch("mg_reset_idx");
}

int mg_hand_finalize(const mg_task_params* tp, const mg_task_buffers* tb, void* stream) {
  if (!tp || !tb || !tb->reduce_scratch || !tb->consecutive_successes)
    return fail(MG_EINVAL, "mg_hand_finalize: needs reduce_scratch and consecutive_successes");
  hipLaunchKernelGGL(k_hand_finalize, dim3(1), dim3(64), 0, (hipStream_t)stream, *tp, *tb);
  return check_launch("mg_hand_finalize");
}

int mg_env_step_replay(mg_sim* sim, const mg_task_params* tp, const mg_task_buffers* tb, const mg_replay* rp,
                       void* stream) {
  if (!rp || !rp->dof_state) return fail(MG_EINVAL, "mg_env_step_replay: bad replay state");
  if (sim && sim->host_model.obj_type && (!rp->root_states || !rp->rigid_body_states))
    return fail(MG_EINVAL, "mg_env_step_replay: hand tasks need root and rigid-body states");
  return env_step(sim, tp, tb, rp, stream);
}


}  // extern "C"
