// migym.hip — C-ABI (include/migym.h) and kernels of the MI355X physics-step +
// observation/reward path.  One lane per actor/env; every kernel is
// asynchronous on the caller's stream; no entry point synchronises.
#include <hip/hip_runtime.h>

#include <new>
#include <string>

#include "../../include/migym.h"
#include "team_physics.hpp"
#include "task.hpp"

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(MG_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
  return MG_OK;
}
constexpr int kBlock = 64;
inline int grid_for(int n) { return (n + kBlock - 1) / kBlock; }
}  // namespace

struct mg_sim {
  mg_model host_model;
  mg_model* d_model;
  mg_sim_params params;
  int32_t n;        // actors
  int32_t device;
  mg_state_views views;
  bool bound;
};

// ------------------------------------------------------------------------------------------------ kernels
// gym.simulate: one team of T lanes per actor (team_physics.hpp)
template <int T, int MN, int MC, int MG, int MP>
__global__ __launch_bounds__(kBlock) void k_simulate(const mg_model* __restrict__ m, mg_sim_params p, int n,
                                                     float* __restrict__ root, float* __restrict__ dof,
                                                     const float* __restrict__ act, float* __restrict__ sensors,
                                                     float* __restrict__ dof_force) {
  constexpr int E = kBlock / T;
  __shared__ mg::TeamLDS<T, MN, MC> lds[E];
  __shared__ mg::ModelTile<MN, MG, MP> tile;
  mg::load_tile(&tile, m);
  __syncthreads();
  const int team = threadIdx.x / T;
  const int a = blockIdx.x * E + team;
  const bool valid = a < n;
  const int ac = valid ? a : n - 1;
  const int nd = m->num_dofs, ns = m->num_sensors;
  mg::Team<T, MN, MC, MG, MP> t;
  t.init(&lds[team], &tile, m, &p);
  __syncthreads();
  t.load(root + (size_t)13 * ac, dof + (size_t)2 * nd * ac, act ? act + (size_t)nd * ac : nullptr);
  for (int st = 0; st < p.substeps; st++) t.substep();
  t.outputs(lds[team].sens, lds[team].dforce);
  t.stage_state();
  __syncthreads();
  if (valid) {
    mg::TeamLDS<T, MN, MC>& L = lds[team];
    if (!m->fixed_base)
      for (int k = t.tl; k < 13; k += T) root[(size_t)13 * a + k] = L.root[k];
    for (int k = t.tl; k < 2 * nd; k += T) dof[(size_t)2 * nd * a + k] = L.dof[k];
    if (sensors)
      for (int k = t.tl; k < 6 * ns; k += T) sensors[(size_t)6 * ns * a + k] = L.sens[k];
    if (dof_force)
      for (int k = t.tl; k < nd; k += T) dof_force[(size_t)nd * a + k] = L.dforce[k];
  }
}

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
                  (uint64_t)(tb.env_offset + a), tb.step_counter, root, dof, &pot, &prev);
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

// The whole VecTask.step for one actor, fused: clamp -> actuation -> simulate -> post_physics.
// One team of T lanes per actor; the team leader (tl == 0) runs the task layer on the LDS-staged
// state, the team writes it back to HBM.  Multi-agent: the agents of an env are consecutive
// teams of one wave, so the AND-filter is a ballot over team leaders and the others-block a
// shuffle from the other agents' leaders.
template <int T, int MN, int MC, int MG, int MP>
__global__ __launch_bounds__(kBlock) void k_env_step(const mg_model* __restrict__ m, mg_sim_params p,
                                                     mg_task_params tp, mg_state_views v, mg_task_buffers tb, int n) {
  constexpr int E = kBlock / T;
  __shared__ mg::TeamLDS<T, MN, MC> lds[E];
  __shared__ mg::ModelTile<MN, MG, MP> tile;
  mg::load_tile(&tile, m);
  __syncthreads();
  const int team = threadIdx.x / T;
  const int a = blockIdx.x * E + team;
  const bool valid = a < n;
  const int ac = valid ? a : n - 1;
  const int na = tp.num_actions, nd = m->num_dofs, ns = m->num_sensors;
  mg::TeamLDS<T, MN, MC>& L = lds[team];
  mg::Team<T, MN, MC, MG, MP> t;
  t.init(&L, &tile, m, &p);
  __syncthreads();
  const int64_t reset_in = tb.reset[ac];
  // pre_physics_step: clamp + effort (ant.py:281-285; humanoid.py:281-285; cartpole.py:159-163)
  t.load(v.root_states + (size_t)13 * ac, v.dof_state + (size_t)2 * nd * ac, nullptr);
  if (t.node > 0) {
    const int d = t.node - 1;
    float tau;
    if (tp.task_id == MG_TASK_CARTPOLE) {
      tau = d == 0 ? mg::clampf(tb.actions[(size_t)na * ac], tp.clip_actions) * tp.power_scale : 0.0f;
    } else {
      const float act = d < na ? mg::clampf(tb.actions[(size_t)na * ac + d], tp.clip_actions) : 0.0f;
      tau = act * tp.motor_effort[d] * tp.power_scale;
    }
    t.tau = tau;
    if (valid && v.dof_actuation) const_cast<float*>(v.dof_actuation)[(size_t)nd * a + d] = tau;
  }
  for (int st = 0; st < p.substeps; st++) t.substep();
  t.outputs(L.sens, L.dforce);
  t.stage_state();
  __syncthreads();

  // ---------------- post_physics_step (ant.py:287-297) on the staged state
  const int A = tp.num_agents > 1 ? tp.num_agents : 1;
  const int k = a % A;
  const float* off = tp.agent_offset[k];
  const int lane = threadIdx.x & 63;
  bool do_reset = reset_in != 0;
  if (A > 1) {  // AND filter over the env's agents (franka_reach_MA.py:875-885)
    const unsigned long long mk = __ballot(t.tl == 0 && valid && reset_in != 0);
    bool all = true;
    for (int j = 0; j < A; j++) all = all && ((mk >> ((team - k + j) * T)) & 1ull);
    do_reset = all;
  }
  float pot = 0.0f, prev = 0.0f, up[3] = {0, 0, 0}, hd[3] = {0, 0, 0};
  int64_t progress = tb.progress[ac] + 1;
  int64_t reset = reset_in;
  float act[64];
  if (t.tl == 0) {
    for (int i = 0; i < na; i++) {
      act[i] = mg::clampf(tb.actions[(size_t)na * ac + i], tp.clip_actions);
      if (valid && tb.actions_out) tb.actions_out[(size_t)na * a + i] = act[i];
    }
    if (tb.potentials) { pot = tb.potentials[ac]; prev = tb.prev_potentials[ac]; }
    if (do_reset) {
      mg::reset_env(&tp, off, tb.noise ? tb.noise + (size_t)2 * nd * ac : nullptr, tb.seed,
                    (uint64_t)(tb.env_offset + a), tb.step_counter, L.root, L.dof, &pot, &prev);
      progress = 0;
      reset = 0;
    }
  }
  __syncthreads();
  const int no = tp.num_obs;
  float* o = tb.obs + (size_t)no * ac;
  if (t.tl == 0 && valid)
    mg::obs_env(&tp, off, L.root, L.dof, L.dforce, L.sens, act, &pot, &prev, up, hd, o);
  if (A > 1) {  // others block, cyclic shift after self (franka_reach_MA.py:604-608)
    const float px = L.root[0], py = L.root[1], pz = L.root[2];
    const int base = no - 3 * (A - 1);
    for (int j = 1; j < A; j++) {
      const int src = (team - k + (k + j) % A) * T;
      const float qx = __shfl(px, src), qy = __shfl(py, src), qz = __shfl(pz, src);
      if (t.tl == 0 && valid) {
        o[base + 3 * (j - 1) + 0] = qx - px;
        o[base + 3 * (j - 1) + 1] = qy - py;
        o[base + 3 * (j - 1) + 2] = qz - pz;
      }
    }
  }
  if (t.tl == 0 && valid) {
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
  }
  __syncthreads();
  if (valid) {  // state write-back (gym layouts), team-cooperative
    if (!m->fixed_base || tp.task_id != MG_TASK_CARTPOLE)
      for (int q = t.tl; q < 13; q += T) v.root_states[(size_t)13 * a + q] = L.root[q];
    for (int q = t.tl; q < 2 * nd; q += T) v.dof_state[(size_t)2 * nd * a + q] = L.dof[q];
    if (v.sensors)
      for (int q = t.tl; q < 6 * ns; q += T) v.sensors[(size_t)6 * ns * a + q] = L.sens[q];
    if (v.dof_force)
      for (int q = t.tl; q < nd; q += T) v.dof_force[(size_t)nd * a + q] = L.dforce[q];
  }
}

__global__ void k_set_indexed(float* __restrict__ dst, const float* __restrict__ src, const int32_t* __restrict__ idx,
                              int nidx, int row) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nidx * row) return;
  const int r = t / row, c = t % row;
  const size_t a = (size_t)idx[r] * row + c;
  dst[a] = src[a];
}

// ------------------------------------------------------------------------------------------------ dispatch
// Kernel instances by capacity: team size T (>= velocity columns, nodes and sensors), nodes MN,
// contacts MC.  The smallest instance that fits the model is launched.
#define MG_INSTANCES(X) \
  X(8, 4, 8, 4, 0) X(16, 9, 16, 16, 0) X(16, 16, 24, 24, 32) X(32, 24, 32, 24, 160) X(32, 32, 48, 48, 192) \
  X(64, 40, 48, 48, 192)

// team size the dispatcher picks for a model (0: none fits)
static int team_size(const mg_model& m, int max_contacts) {
  const int nv = (m.fixed_base ? 0 : 6) + m.num_dofs;
  const int lanes = nv > m.num_sensors ? nv : m.num_sensors;
#define MG_T(T, MN, MC, MG, MP)                                                                 \
  if (m.num_nodes <= MN && max_contacts <= MC && lanes <= T && (m.fixed_base || T >= 6) &&        \
      m.num_geoms <= MG && m.num_pairs <= MP)                                                      \
    return T;
  MG_INSTANCES(MG_T)
#undef MG_T
  return 0;
}

template <template <int, int, int, int, int> class F, typename... A>
static int dispatch(const mg_model& m, int max_contacts, A... args) {
  const int nv = (m.fixed_base ? 0 : 6) + m.num_dofs;
  const int lanes = nv > m.num_sensors ? nv : m.num_sensors;
#define MG_TRY(T, MN, MC, MG, MP)                                                              \
  if (m.num_nodes <= MN && max_contacts <= MC && lanes <= T && (m.fixed_base || T >= 6) &&       \
      m.num_geoms <= MG && m.num_pairs <= MP) {                                                   \
    F<T, MN, MC, MG, MP>::run(args...);                                                          \
    return MG_OK;                                                                                 \
  }
  MG_INSTANCES(MG_TRY)
#undef MG_TRY
  return fail(MG_ECAPACITY, "model exceeds the largest kernel instance");
}

template <int T, int MN, int MC, int MG, int MP>
struct RunSimulate {
  static void run(hipStream_t s, const mg_sim* sim) {
    const mg_state_views& v = sim->views;
    const int E = kBlock / T;
    hipLaunchKernelGGL((k_simulate<T, MN, MC, MG, MP>), dim3((sim->n + E - 1) / E), dim3(kBlock), 0, s, sim->d_model,
                       sim->params, sim->n, v.root_states, v.dof_state, v.dof_actuation, v.sensors, v.dof_force);
  }
};
template <int T, int MN, int MC, int MG, int MP>
struct RunEnvStep {
  static void run(hipStream_t s, const mg_sim* sim, const mg_task_params* tp, const mg_task_buffers* tb) {
    const int E = kBlock / T;
    hipLaunchKernelGGL((k_env_step<T, MN, MC, MG, MP>), dim3((sim->n + E - 1) / E), dim3(kBlock), 0, s, sim->d_model,
                       sim->params, *tp, sim->views, *tb, sim->n);
  }
};

// ------------------------------------------------------------------------------------------------ C ABI
extern "C" {

const char* mg_last_error(void) { return g_err.c_str(); }
int mg_version(void) { return MG_VERSION; }
size_t mg_model_sizeof(void) { return sizeof(mg_model); }
size_t mg_task_params_sizeof(void) { return sizeof(mg_task_params); }
size_t mg_task_buffers_sizeof(void) { return sizeof(mg_task_buffers); }
size_t mg_sim_params_sizeof(void) { return sizeof(mg_sim_params); }
size_t mg_state_views_sizeof(void) { return sizeof(mg_state_views); }

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
  *out = s;
  return MG_OK;
}

int mg_sim_bind(mg_sim* sim, const mg_state_views* views) {
  if (!sim || !views || !views->root_states || !views->dof_state) return fail(MG_EINVAL, "mg_sim_bind: bad views");
  if (sim->host_model.num_sensors > 0 && !views->sensors)
    return fail(MG_EINVAL, "mg_sim_bind: model has force sensors but no sensor buffer");
  sim->views = *views;
  sim->bound = true;
  return MG_OK;
}

int mg_sim_simulate(mg_sim* sim, void* stream) {
  if (!sim || !sim->bound) return fail(MG_EINVAL, "mg_sim_simulate: sim not bound");
  int rc = dispatch<RunSimulate>(sim->host_model, sim->params.max_contacts, (hipStream_t)stream,
                                 (const mg_sim*)sim);
  if (rc) return rc;
  return check_launch("mg_sim_simulate");
}

int mg_sim_destroy(mg_sim* sim) {
  if (!sim) return MG_OK;
  (void)hipFree(sim->d_model);
  delete sim;
  return MG_OK;
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
  } else {
    return fail(MG_EINVAL, "mg_set_indexed: unknown target");
  }
  if (dst == src) return MG_OK;  // caller wrote into the bound buffer itself (gym views alias sim memory)
  const int total = n * row;
  hipLaunchKernelGGL(k_set_indexed, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream, dst, src, idx, n,
                     row);
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

int mg_post_physics(mg_sim* sim, const mg_task_params* tp, const mg_state_views* views, const mg_task_buffers* tb,
                    int32_t n, void* stream) {
  if (!tp || !tb) return fail(MG_EINVAL, "mg_post_physics: bad args");
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
  hipLaunchKernelGGL(k_post_physics, dim3(grid_for(n)), dim3(kBlock), 0, (hipStream_t)stream, *tp, v, *tb, n);
  return check_launch("mg_post_physics");
}

int mg_env_step(mg_sim* sim, const mg_task_params* tp, const mg_task_buffers* tb, void* stream) {
  if (!sim || !sim->bound || !tp || !tb || !tb->actions || !tb->obs || !tb->rew || !tb->reset || !tb->progress ||
      !tb->timeout)
    return fail(MG_EINVAL, "mg_env_step: bad arguments");
  if (tp->task_id != MG_TASK_CARTPOLE && (!tb->potentials || !tb->prev_potentials || !tb->up_vec || !tb->heading_vec))
    return fail(MG_EINVAL, "mg_env_step: locomotion task needs potential/up/heading buffers");
  if (tp->num_actions > sim->host_model.num_nodes && tp->task_id != MG_TASK_CARTPOLE)
    return fail(MG_EINVAL, "mg_env_step: more actions than DOFs");
  if (tp->num_agents > 1) {
    // the agents of an env must be teams of one wave (ballot/shuffle exchange): A | 64/T
    const int T = team_size(sim->host_model, sim->params.max_contacts);
    if (T == 0 || tp->num_agents > MG_MAX_AGENTS || (64 / T) % tp->num_agents != 0 ||
        sim->n % tp->num_agents != 0)
      return fail(MG_EINVAL, "mg_env_step: num_agents must divide the envs per wave (64 / team size) "
                             "and the actor count");
  }
  int rc = dispatch<RunEnvStep>(sim->host_model, sim->params.max_contacts, (hipStream_t)stream, (const mg_sim*)sim,
                                tp, tb);
  if (rc) return rc;
  return check_launch("mg_env_step");
}

}  // extern "C"
