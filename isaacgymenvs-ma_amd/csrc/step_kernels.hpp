// step_kernels.hpp — the team kernels of the hot path (one team of T lanes per actor):
//   k_simulate   gym.simulate alone
//   k_env_step   the whole VecTask.step of the locomotion tasks (Ant, Humanoid, Cartpole, MA-Ant)
//   k_hand_step  the whole VecTask.step of ShadowHand
// plus the host launchers RunSimulate / RunEnvStep (dispatch.hpp).  Included only by inst.hip, which
// instantiates one capacity instance per translation unit.
#pragma once
#include <new>

#include "dispatch.hpp"
#include "hand_task.hpp"
#include "task.hpp"
#include "team_physics.hpp"


// waves per SIMD the register allocator targets (2: the 256-VGPR budget; an A/B variant may ask for 3, <= 168 VGPRs)
#ifndef MG_WAVES_PER_EU
#define MG_WAVES_PER_EU 2
#endif
// ... and for the instances with the compact team layout (mg::TeamLDSC: Ant, MA-Ant), whose LDS holds 12 waves per CU
#ifndef MG_WAVES_COMPACT
#define MG_WAVES_COMPACT 3
#endif
// the compact 32-lane instances (Humanoid) on the static grid too (1) or on the work queue (0)
#ifndef MG_COMPACT_STATIC32
#define MG_COMPACT_STATIC32 0
#endif
// dynamic LDS added to every step-kernel launch (0; an occupancy A/B variant pads it to hold fewer waves per CU)
// an explicit VGPR budget for k_env_step (0: the waves_per_eu budget); register-pressure experiments only
#ifndef MG_NUM_VGPR
#define MG_NUM_VGPR 0
#endif
#if MG_NUM_VGPR
#define MG_VGPR_ATTR __attribute__((amdgpu_num_vgpr(MG_NUM_VGPR)))
#else
#define MG_VGPR_ATTR
#endif
#ifndef MG_LDS_PAD
#define MG_LDS_PAD 0
#endif
// the locomotion observation head on four team lanes (mg::obs_head_team) instead of the leader (0: mg::obs_head)
// the locomotion task layer's per-env scalars (progress, potentials) loaded at the start of the step (0: after it)
#ifndef MG_TASK_PREFETCH
#define MG_TASK_PREFETCH 1
#endif
#ifndef MG_TEAM_OBS_HEAD
#define MG_TEAM_OBS_HEAD 1
#endif

namespace mgi {
#ifdef MG_PHASE_TIMING
// per-wave accumulators (one row of MG_NUM_PHASES per block; plain read-modify-writes by the block's own wave,
// so the profiling build adds no atomic traffic that would slow the solver's memory path)
constexpr int kPhaseCap = 1 << 16;  // waves tracked
// one copy per instance translation unit (each is its own code object): phase_buf_publish<I> sets it
static __device__ unsigned long long* g_phase_buf;
#define MG_PHASE_FLUSH(t, item)                                                        \
  {                                                                                    \
    const unsigned gw_ = (unsigned)(item), l_ = threadIdx.x & 63;                      \
    if (g_phase_buf && gw_ < kPhaseCap && l_ < MG_NUM_PHASES) {                        \
      unsigned int v_ = 0;                                                             \
      for (int i_ = 0; i_ < MG_NUM_PHASES; i_++)                                       \
        if ((int)l_ == i_) v_ = (t).ph[i_];                                            \
      g_phase_buf[MG_NUM_PHASES * (size_t)gw_ + l_] += v_;                             \
    }                                                                                  \
  }
#else
#define MG_PHASE_FLUSH(t, item)
#endif

// ------------------------------------------------------------------------------------------------ launch shape
// Waves per block W.  A block's W waves share one LDS model tile (each team's own LDS is per wave), so a
// larger W leaves more of the CU's 160 KB LDS for resident waves; a smaller W lets the CU refill sooner
// when a wave finishes (a block's slots free only when its slowest wave is done).  W is the smallest
// of 1, 2, 4, 8 that reaches the most resident waves per CU (at most 4 x the instance's waves per SIMD: 8 at the
// 256-register budget, 12 at 168).
template <int T, int MN, int MC, int MG, int MP, int OBJ, bool DR, int LAY = 0>
struct Shape {
  using TL = mg::TeamLDSOf<T, MN, MC, OBJ, MG, MP, LAY>;
  static constexpr int E1 = 64 / T;  // teams (actors) per wave
  static constexpr size_t kTile = sizeof(mg::ModelTile<MN, MG, MP, mg::tile_hull_verts(OBJ)>);
  static constexpr size_t kWave = E1 * (sizeof(mg::BankSlot<TL, T>) + (DR ? sizeof(mg::DrTile<MN, MG>) : 0));
  static constexpr int fit(int w, int cap) {  // resident waves per CU with w-wave blocks, at most cap
    const size_t blk = (kTile + w * kWave + 511) / 512 * 512;
    const int b = (int)((160 * 1024) / blk);
    return b * w < cap ? b * w : cap;
  }
  // waves per SIMD of the instance (the register budget: 2 -> 256 VGPRs, 3 -> 168): 3 for the compact layouts whose
  // LDS holds twelve waves per CU with some block width (Ant, MA-Ant, Humanoid), else 2
  static constexpr bool fits12() { return fit(1, 12) >= 12 || fit(2, 12) >= 12 || fit(4, 12) >= 12 || fit(8, 12) >= 12; }
  static constexpr int kWPE = (TL::kCompact && !DR && fits12()) ? MG_WAVES_COMPACT : MG_WAVES_PER_EU;
  static constexpr int kMaxWaves = 4 * kWPE;
  static constexpr int per_cu(int w) { return fit(w, kMaxWaves); }
  static constexpr int pick() {
    int best = 1;
    for (int w = 2; w <= 8; w *= 2)
      if (per_cu(w) > per_cu(best)) best = w;
    return best;
  }
  static constexpr int W = pick();
  static constexpr int kThreads = 64 * W;
  static constexpr int E = E1 * W;  // teams per block
  static_assert(per_cu(W) >= 1, "one block must fit the CU's LDS");
  // one work item per wave on a static grid (no work queue): the one-wave blocks, and the compact instances'
  // two-wave blocks (a block's waves hold envs of like cost under the sort, so little of its LDS waits on a slower
  // partner, and the queue's loop costs registers at the 168-VGPR budget)
  static constexpr bool kStatic = W == 1 || (TL::kCompact && (T == 16 || MG_COMPACT_STATIC32));
};

// ------------------------------------------------------------------------------------------------ work queue
// The step kernels launch the resident capacity (as many blocks as the CUs hold at once, launch_wq) and
// each wave loops over work items (one item = the E1 teams of one wave): its own index in the grid first,
// then items dequeued from a device counter until they run out.  A CU thus refills a wave's slot as soon
// as that wave is done; with one block per W waves launched over the whole batch, a block's LDS stays held
// until its slowest wave finishes (Humanoid: 4-wave blocks, 23 % of the wave slots idle),
// and the model tile is copied once per resident block instead of once per W waves of work.
// wq[0] counts dequeues, wq[1] finished waves; the last wave to finish zeroes both (every other wave has
// made its final dequeue before its wq[1] add), so the next launch on the stream starts from zero.
// a zero the compiler cannot see through, redrawn per work item: every address of the item's body is offset by it,
// so nothing the body loads (LDS tile, model, kernel arguments) is hoisted out of the work loop and kept in
// registers across all items (that hoisting took the Ant kernel from 11 to 107 spilled registers)
__device__ __forceinline__ int opaque_zero() {
  int z = 0;
  asm volatile("" : "+s"(z));
  return z;
}
__device__ __forceinline__ int wq_next(unsigned* wq, int grid_waves) {
  unsigned v = 0u;
  if ((threadIdx.x & 63) == 0) v = atomicAdd(&wq[0], 1u);
  return grid_waves + (int)__builtin_amdgcn_readfirstlane(v);
}
// kernel span (mg_kernel_span_begin): lane 0 of each wave stores its start and end times (GPU wall clock) into the
// wave's own pair of the launch's slot -- plain stores to distinct addresses, no atomics (a same-address atomic per
// wave cost Ant 12 % in its first form); mg_kernel_span_read reduces them.  A kernel-argument branch otherwise.
// (MG_NO_SPAN: compiled out, the A/B variant that checks the hooks cost the timed launches nothing)
__device__ __forceinline__ void span_start(unsigned long long* clk, int wave) {
#ifndef MG_NO_SPAN
  if (clk && (threadIdx.x & 63) == 0) clk[2 * (size_t)wave] = (unsigned long long)wall_clock64();
#endif
}
__device__ __forceinline__ void span_end(unsigned long long* clk, int wave) {
#ifndef MG_NO_SPAN
  if (clk && (threadIdx.x & 63) == 0) clk[2 * (size_t)wave + 1] = (unsigned long long)wall_clock64();
#endif
}
// sort: block 0 zeroes the bin totals this launch's permutation was built from (k_oscatter, their last reader, has
// finished: stream order), so every sort starts from zero and the launches hold no host-side parity (graph replays)
__device__ __forceinline__ void sort_totals_clear(const MgOrder& ord) {
  if (ord.tot_clear && blockIdx.x == 0)
    for (int i = (int)threadIdx.x; i < kSortTot; i += (int)blockDim.x) ord.tot_clear[i] = 0u;
}
__device__ __forceinline__ void wq_done(unsigned* wq, int grid_waves) {
  if ((threadIdx.x & 63) == 0 && atomicAdd(&wq[1], 1u) == (unsigned)grid_waves - 1u) {
    atomicExch(&wq[0], 0u);
    atomicExch(&wq[1], 0u);
  }
}

// ------------------------------------------------------------------------------------------------ kernels
// gym.simulate: one team of T lanes per actor (team_physics.hpp).  OBJ: hand-task envs with root
// rows [articulation, object, goal], PD targets and rigid-body rows [bodies..., object, goal].
template <int T, int MN, int MC, int MG, int MP, int OBJ, bool DR, bool TGS = false, int LAY = 0>
__global__ __launch_bounds__((Shape<T, MN, MC, MG, MP, OBJ, DR, LAY>::kThreads)) __attribute__((amdgpu_waves_per_eu(Shape<T, MN, MC, MG, MP, OBJ, DR, LAY>::kWPE))) void k_simulate(
    const mg_model* __restrict__ m, const void* __restrict__ timg, mg_sim_params p, mg_state_views v, int n) {
  using SH = Shape<T, MN, MC, MG, MP, OBJ, DR, LAY>;
  constexpr int E = SH::E, W = SH::W;
  constexpr int ROWS = OBJ ? 3 : 1;
  __shared__ mg::BankSlot<mg::TeamLDSOf<T, MN, MC, OBJ, MG, MP, LAY>, T> lds[E];
  __shared__ typename mg::Team<T, MN, MC, MG, MP, OBJ>::MT tile;
  __shared__ mg::DrTile<DR ? MN : 1, DR ? MG : 1> drt[DR ? E : 1];
  mg::copy_tile(&tile, static_cast<const typename mg::Team<T, MN, MC, MG, MP, OBJ>::MT*>(timg));
  __syncthreads();  // the only block-wide barrier: every later phase synchronises its own wave
  const int team = threadIdx.x / T;
  const int a = blockIdx.x * E + team;
  const bool valid = a < n;
  const int ac = valid ? a : n - 1;
  const int nd = m->num_dofs, ns = m->num_sensors;
  mg::Team<T, MN, MC, MG, MP, OBJ, TGS, LAY> t;
  t.init(&lds[team].v, &tile, m, &p);
  if constexpr (DR) {  // domain randomization: this actor's env_props row into the team's DrTile
    mg::load_dr<T>(&drt[team], v.env_props + (size_t)v.env_props_stride * ac, m, t.tl);
    t.drn = &drt[team].node[0][0];
    t.drg = drt[team].geom;
    t.drt = &drt[team].ten[0][0];
    t.dro = drt[team].obj;
  }
  if (OBJ && t.tl < 4) {  // applied force on the object row of rb_forces (apply_rigid_body_force_tensors)
    const float* fr = v.rb_forces ? v.rb_forces + ((size_t)(m->num_bodies + 2) * ac + m->num_bodies) * 3 : nullptr;
    lds[team].v.oforce[t.tl] = t.tl < 3 ? (fr ? fr[t.tl] : 0.0f) : (v.rb_force_space == MG_LOCAL_SPACE ? 1.0f : 0.0f);
  }
  mg::wsync();
  float* root = v.root_states + (size_t)13 * ROWS * ac;
  t.load(root, v.dof_state + (size_t)2 * nd * ac, v.dof_actuation ? v.dof_actuation + (size_t)nd * ac : nullptr,
         OBJ ? root + 13 : nullptr, v.dof_targets ? v.dof_targets + (size_t)nd * ac : nullptr);
  for (int st = 0; st < p.substeps; st++) t.substep();
  t.outputs(lds[team].v.st().sens, lds[team].v.st().dforce,
            (valid && v.net_contact_forces) ? v.net_contact_forces + (size_t)3 * (m->num_bodies + (OBJ ? 2 : 0)) * a
                                            : nullptr);
  t.stage_state();
  mg::wsync();
  if (valid) {
    auto& L = lds[team].v;
    if (!m->fixed_base)
      for (int k = t.tl; k < 13; k += T) root[k] = L.st().root[k];
    if (OBJ)
      for (int k = t.tl; k < 13; k += T) root[13 + k] = L.oroot[k];
    for (int k = t.tl; k < 2 * nd; k += T) v.dof_state[(size_t)2 * nd * a + k] = L.st().dof[k];
    if (v.sensors)
      for (int k = t.tl; k < 6 * ns; k += T) v.sensors[(size_t)6 * ns * a + k] = L.st().sens[k];
    if (v.dof_force)
      for (int k = t.tl; k < nd; k += T) v.dof_force[(size_t)nd * a + k] = L.st().dforce[k];
    if (v.rigid_body_states) {
      const int nb = m->num_bodies, nbe = nb + (OBJ ? 2 : 0);
      float* rb = v.rigid_body_states + (size_t)13 * nbe * a;
      for (int b = t.tl; b < nb; b += T) t.body_state(b, rb + 13 * b);
      if (OBJ)
        for (int k = t.tl; k < 26; k += T) rb[13 * nb + k] = k < 13 ? L.oroot[k] : root[26 + k - 13];
    }
  }
}

// The whole VecTask.step for one actor, fused: clamp -> actuation -> simulate -> post_physics.
// One team of T lanes per actor; the team leader (tl == 0) runs the task layer on the LDS-staged
// state, the team writes it back to HBM.  Multi-agent: the agents of an env are consecutive
// teams of one wave, so the AND-filter is a ballot over team leaders and the others-block a
// shuffle from the other agents' leaders.
// amdgpu_waves_per_eu(MG_WAVES_PER_EU): the register budget that lets two waves share a SIMD (the team kernels
// are latency-bound; occupancy is the lever — DESIGN.md §3)
// RP: physics-bypass replay instance (mg_env_step_replay): the task layer below runs unchanged on the
// post-simulate state `rp` supplies instead of the substeps (tests only; never the bench path).
// the actor a team slot works on: the slot itself, or under a work ordering (MgOrder, sim->order_mode) the env at
// the slot's position in the sort's permutation, or in the previous launch's bucket lists, heaviest bucket first (envs of A agents stay whole and
// aligned: the AND filter and the "others" block exchange within the env's A consecutive teams of one wave).  The
// wave's lanes 0..kOrderBuckets-1 load the counts and scan them; each lane finds its position's bucket through the
// wave-uniform prefixes.
__device__ __forceinline__ int ordered_actor(const MgOrder& ord, int slot, int n, int A) {
  const int a1 = A > 1 ? A : 1;
  if (ord.order) {  // sort: the permutation k_oscatter wrote (of units of ord.unit consecutive actors)
    const int s = slot < n ? slot : n - 1;
    return ord.order[s / ord.unit] * ord.unit + s % ord.unit;
  }
  if (!ord.rcnt) return slot < n ? slot : n - 1;
  const int lane = (int)(threadIdx.x & 63);
  unsigned inc = lane < kOrderBuckets ? ord.rcnt[lane] : 0u;
#pragma unroll
  for (int d = 1; d < kOrderBuckets; d <<= 1) {
    const unsigned y = __shfl_up(inc, d);
    inc += lane >= d ? y : 0u;
  }
  const unsigned p = (unsigned)((slot < n ? slot : n - 1) / a1);
  unsigned b = 0u, base = 0u;
#pragma unroll
  for (int j = 0; j < kOrderBuckets; j++) {
    const unsigned v = (unsigned)__builtin_amdgcn_readlane((int)inc, j);
    b += v <= p ? 1u : 0u;
    base = v <= p ? v : base;
  }
  b = b < (unsigned)kOrderBuckets ? b : (unsigned)kOrderBuckets - 1u;
  return ord.rlist[(size_t)b * ord.cap + (p - base)] * a1 + (slot < n ? slot : n - 1) % a1;
}
// the bucket of an env whose step used `rows` constraint rows (descending: the heaviest first)
__device__ __forceinline__ int order_bucket(int rows) {
  const int c = rows / kOrderWidth;
  return kOrderBuckets - 1 - (c < kOrderBuckets - 1 ? c : kOrderBuckets - 1);
}
// the next launch's lists: env unit u (of this launch's step) appended to the bucket of its row count
__device__ __forceinline__ void order_append(const MgOrder& ord, int rows, int u) {
  const int b = order_bucket(rows);
  const unsigned k = atomicAdd(&ord.wcnt[b], 1u);
  if (k < (unsigned)ord.cap) ord.wlist[(size_t)b * ord.cap + k] = u;  // always, unless the counts were not cleared
}
// every wave of an ordered launch checks out; the last one clears the counts the launch read (every wave has read
// them: it started before the last one finished) and the counter, for the launch after next
__device__ __forceinline__ void order_done(const MgOrder& ord, int grid_waves) {
  if (ord.wcnt && (threadIdx.x & 63) == 0 && atomicAdd(ord.done, 1u) == (unsigned)grid_waves - 1u) {
    for (int b = 0; b < kOrderBuckets; b++) atomicExch(&ord.rclear[b], 0u);
    atomicExch(ord.done, 0u);
  }
}

// one work item of k_env_step: the E1 teams of one wave (item = the wave's global index)
template <int T, int MN, int MC, int MG, int MP, bool DR, bool RP, bool TGS = false, int LAY = 0>
__device__ __forceinline__ void env_step_item(
    const mg_model* __restrict__ m, const mg::ModelTile<MN, MG, MP>& tile, mg::BankSlot<mg::TeamLDSOf<T, MN, MC, 0, MG, MP, LAY>, T>* lds,
    mg::DrTile<DR ? MN : 1, DR ? MG : 1>* drt, const mg_sim_params& p, const mg_task_params& tp, const mg_state_views& v,
    const mg_task_buffers& tb, int n, const mg_replay& rp, int item, const MgOrder& ord) {
  using SH = Shape<T, MN, MC, MG, MP, 0, DR, LAY>;
  const int team = threadIdx.x / T;
  const int wt = (threadIdx.x & 63) / T;  // team index within the wave (ballot / shuffle positions)
  const int slot = item * SH::E1 + wt;
  const bool valid = slot < n;
  const int a = ordered_actor(ord, slot, n, tp.num_agents);
  const int ac = valid ? a : n - 1;
  const int na = tp.num_actions, nd = m->num_dofs, ns = m->num_sensors;
  mg::TeamLDSOf<T, MN, MC, 0, MG, MP, LAY>& L = lds[team].v;
  mg::Team<T, MN, MC, MG, MP, 0, TGS, LAY> t;
  t.init(&L, &tile, m, &p, SH::W > 1);
  if constexpr (DR) {  // domain randomization: this actor's env_props row into the team's DrTile
    mg::load_dr<T>(&drt[team], v.env_props + (size_t)v.env_props_stride * ac, m, t.tl);
    t.drn = &drt[team].node[0][0];
    t.drg = drt[team].geom;
    t.drt = &drt[team].ten[0][0];
    t.dro = drt[team].obj;
  }
  mg::wsync();
  const int64_t reset_in = tb.reset[ac];
  // the task layer's per-env scalars, loaded now so that their latency hides under the physics (nothing in the
  // step writes them before the task layer does); not for the compact 16-lane kernel, whose 168 registers it costs
  // (profiles/r06/ab_task_prefetch.txt: Ant 65,536 -0.3 %, MA-Ant -0.4 %; Humanoid +0.6 %, Ant 8,192 +0.9 %)
  constexpr bool kTaskPf = MG_TASK_PREFETCH && !(SH::TL::kCompact && T == 16);
  int64_t progress_in = 0;
  float pot_in = 0.0f, prev_in = 0.0f;
  if constexpr (kTaskPf) {
    progress_in = tb.progress[ac];
    pot_in = tb.potentials ? tb.potentials[ac] : 0.0f;
    prev_in = tb.potentials ? tb.prev_potentials[ac] : 0.0f;
  }
  t.ph_start();
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
  t.ph_mark(14);
  if constexpr (RP) {  // gym.simulate replaced by the injected post-simulate state
    const float* rr = rp.root_states ? rp.root_states : v.root_states;
    for (int q = t.tl; q < 13; q += T) L.st().root[q] = rr[(size_t)13 * ac + q];
    for (int q = t.tl; q < 2 * nd; q += T) L.st().dof[q] = rp.dof_state[(size_t)2 * nd * ac + q];
    for (int q = t.tl; q < 6 * ns; q += T) L.st().sens[q] = rp.sensors ? rp.sensors[(size_t)6 * ns * ac + q] : 0.0f;
    for (int q = t.tl; q < nd; q += T) L.st().dforce[q] = rp.dof_force ? rp.dof_force[(size_t)nd * ac + q] : 0.0f;
  } else {
    // controlFrequencyInv: gym.simulate x cfi between one pre- and one post_physics_step (vec_task.py:381-384)
    const int nsub = p.substeps * (tp.control_freq_inv > 1 ? tp.control_freq_inv : 1);
    for (int st = 0; st < nsub; st++) t.substep();
    // no rigid-body states here: pose-only FK; DOF forces only where something reads them (the bound view, or the
    // Humanoid's observation: the reference's Ant and Cartpole never acquire a DOF-force tensor)
    t.template outputs<true>(L.st().sens,
                             (v.dof_force || tp.task_id == MG_TASK_HUMANOID) ? L.st().dforce : nullptr,
                             (valid && v.net_contact_forces) ? v.net_contact_forces + (size_t)3 * m->num_bodies * a : nullptr);
    t.stage_state();
  }
  mg::wsync();
  t.ph_mark(8);

  // ---------------- post_physics_step (ant.py:287-297) on the staged state
  const int A = tp.num_agents > 1 ? tp.num_agents : 1;
  const int k = a % A;
  const float* off = tp.agent_offset[k];
  bool do_reset = reset_in != 0;
  if (A > 1) {  // AND filter over the env's agents (franka_reach_MA.py:875-885)
    const unsigned long long mk = __ballot(t.tl == 0 && valid && reset_in != 0);
    bool all = true;
    for (int j = 0; j < A; j++) all = all && ((mk >> ((wt - k + j) * T)) & 1ull);
    do_reset = all;
  }
  float pot = 0.0f, prev = 0.0f, up[3] = {0, 0, 0}, hd[3] = {0, 0, 0};
  int64_t progress = (kTaskPf ? progress_in : tb.progress[ac]) + 1;
  int64_t reset = reset_in;
  // self.actions: one lane per action column (na <= T, checked by mg_env_step)
  const bool alane = t.tl < na;
  const float act_l = alane ? mg::clampf(tb.actions[(size_t)na * ac + t.tl], tp.clip_actions) : 0.0f;
  if (valid && alane && tb.actions_out) tb.actions_out[(size_t)na * a + t.tl] = act_l;
  if (tb.potentials) {
    if constexpr (kTaskPf) { pot = pot_in; prev = prev_in; }
    else { pot = tb.potentials[ac]; prev = tb.prev_potentials[ac]; }
  }
  if (do_reset) {  // reset_idx: one lane per DOF draws its noise; the leader resets root and potentials
    const float* nz = tb.noise ? tb.noise + (size_t)2 * nd * ac : nullptr;
    for (int i = t.tl; i < nd; i += T)
      mg::reset_dof(&tp, i, nd, nz, tb.seed, (uint64_t)(tb.env_offset * A + a), tb.step_counter, L.st().dof);
    if (t.tl == 0) mg::reset_root(&tp, off, L.st().root, &pot, &prev);
    progress = 0;
    reset = 0;
  }
  mg::wsync();
  // NaN guard: an actor whose state is not finite after the step gets reset = 1 (every agent
  // of its env under MA layouts, so the AND filter resets the env in the next step), reward 0 and a zero
  // observation row: no NaN reaches the policy, and the next step's masked reset_idx restores it
  bool nf = false;
  for (int q = t.tl; q < (m->fixed_base ? 7 : 13); q += T) nf = nf || !isfinite(L.st().root[q]);
  for (int q = t.tl; q < 2 * nd; q += T) nf = nf || !isfinite(L.st().dof[q]);
  const unsigned long long nfm = __ballot(nf);
  bool bad = false;
  for (int j = 0; j < A; j++) bad = bad || ((nfm >> ((wt - k + j) * T)) & mg::team_bits<T>()) != 0ull;
  // observations staged in the row storage (dead after outputs()), then stored coalesced
  const int no = tp.num_obs;
  float* ost = L.obs_stage();
  if (tp.task_id == MG_TASK_CARTPOLE) {
    if (t.tl < 4) ost[t.tl] = L.st().dof[t.tl];
  } else {
#if MG_TEAM_OBS_HEAD
    mg::obs_head_team(&tp, off, L.st().root, t.tl, t.tb, &pot, &prev, up, hd, ost);  // lanes 0..3, T >= 16
#else
    if (t.tl == 0) mg::obs_head(&tp, off, L.st().root, &pot, &prev, up, hd, ost);
#endif
    const bool hum = tp.task_id == MG_TASK_HUMANOID;
    for (int q = t.tl; q < nd; q += T) {
      ost[12 + q] = mg::t_unscale(L.st().dof[2 * q], tp.dof_lower[q], tp.dof_upper[q]);
      ost[12 + nd + q] = L.st().dof[2 * q + 1] * tp.dof_vel_scale;
      if (hum) ost[12 + 2 * nd + q] = L.st().dforce[q] * tp.contact_force_scale;
    }
    const int bs = 12 + (hum ? 3 : 2) * nd, nss = mg::t_sensors(&tp);
    for (int q = t.tl; q < 6 * nss; q += T) ost[bs + q] = L.st().sens[q] * tp.contact_force_scale;
    if (alane) ost[bs + 6 * nss + t.tl] = act_l;
  }
  if (A > 1) {  // others block, cyclic shift after self (franka_reach_MA.py:604-608)
    const float px = L.st().root[0], py = L.st().root[1], pz = L.st().root[2];
    const int base = no - 3 * (A - 1);
    {  // lane j - 1 of the team writes agent j's three entries (one shuffle per coordinate, per-lane sources)
      const int j = t.tl + 1 < A ? t.tl + 1 : 0;
      const int src = (wt - k + (k + j) % A) * T;
      const float qx = __shfl(px, src), qy = __shfl(py, src), qz = __shfl(pz, src);
      if (t.tl + 1 < A) {
        ost[base + 3 * (j - 1) + 0] = qx - px;
        ost[base + 3 * (j - 1) + 1] = qy - py;
        ost[base + 3 * (j - 1) + 2] = qz - pz;
      }
    }
  }
  mg::wsync();
  // reward: per-action terms as team sums (DPP), the rest on the leader
  float rew = 0.0f;
  if (tp.task_id == MG_TASK_CARTPOLE) {
    if (t.tl == 0) mg::reward_env(&tp, ost, &act_l, pot, prev, progress, &reset, &rew);
  } else {
    float ac2 = act_l * act_l, el = 0.0f, lim = 0.0f;
    if (alane) {
      if (tp.task_id == MG_TASK_ANT) {
        el = fabsf(act_l * ost[12 + nd + t.tl]);
        lim = ost[12 + t.tl] > 0.99f ? 1.0f : 0.0f;
      } else {
        const float ratio = tp.motor_effort[t.tl] / tp.max_motor_effort;
        const float ab = fabsf(ost[12 + t.tl]);
        const float scaled = tp.joints_at_limit_cost_scale * (ab - 0.98f) / 0.02f;
        lim = (ab > 0.98f ? 1.0f : 0.0f) * scaled * ratio;
        el = fabsf(act_l * ost[12 + nd + t.tl]) * ratio;
      }
    }
    ac2 = mg::team_sum<T>(ac2, t.tb);
    el = mg::team_sum<T>(el, t.tb);
    lim = mg::team_sum<T>(lim, t.tb);
    if (tp.task_id == MG_TASK_ANT) lim = lim * tp.joints_at_limit_cost_scale;
    if (t.tl == 0) mg::reward_from_sums(&tp, ost, ac2, el, lim, pot, prev, progress, &reset, &rew);
  }
  if (bad) {
    reset = 1;
    rew = 0.0f;
  }
  if (t.tl == 0 && valid) {
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
  }
  if (valid) {
    float* o = tb.obs + (size_t)no * a;
    for (int q = t.tl; q < no; q += T) {
      const float x = bad ? 0.0f : ost[q];
      o[q] = x;
      if (tb.obs_clamped) tb.obs_clamped[(size_t)no * a + q] = mg::clampf(x, tp.clip_obs);
    }
    if (tb.out_pack) {  // the gather's message row [clamped obs | rew | reset] (migym/dist.py)
      float* pk = tb.out_pack + (size_t)(no + 2) * a;
      for (int q = t.tl; q < no; q += T) pk[q] = bad ? 0.0f : mg::clampf(ost[q], tp.clip_obs);
      if (t.tl == 0) { pk[no] = rew; pk[no + 1] = (float)reset; }
    }
  }
  mg::wsync();
  if (valid) {  // state write-back (gym layouts), team-cooperative
    if (!m->fixed_base || tp.task_id != MG_TASK_CARTPOLE)
      for (int q = t.tl; q < 13; q += T) v.root_states[(size_t)13 * a + q] = L.st().root[q];
    for (int q = t.tl; q < 2 * nd; q += T) v.dof_state[(size_t)2 * nd * a + q] = L.st().dof[q];
    if (v.sensors)
      for (int q = t.tl; q < 6 * ns; q += T) v.sensors[(size_t)6 * ns * a + q] = L.st().sens[q];
    if (v.dof_force)
      for (int q = t.tl; q < nd; q += T) v.dof_force[(size_t)nd * a + q] = L.st().dforce[q];
  }
  if (ord.wcnt || ord.cost) {  // the next launch's order: the unit's largest row count (an env's agents, a wave's envs)
    int rows = L.nrows;
    const int A = tp.num_agents > 1 ? tp.num_agents : 1;
    const int U = ord.wcnt ? A : ord.unit;
    if (U > 1) {
      const int k0 = wt - wt % U;  // the unit's first team in the wave
      for (int k = 0; k < U; k++) rows = max(rows, __shfl(rows, (k0 + k) * T));
    }
    if (valid && t.tl == 0 && a % U == 0) {
      if (ord.wcnt) order_append(ord, rows, a / A);
      else ord.cost[a / U] = (unsigned char)(rows < 255 ? rows : 255);
    }
  }
  t.ph_mark(9);
  MG_PHASE_FLUSH(t, item)
}

template <int T, int MN, int MC, int MG, int MP, bool DR, bool RP, bool TGS = false, int LAY = 0>
__global__ __launch_bounds__((Shape<T, MN, MC, MG, MP, 0, DR, LAY>::kThreads)) __attribute__((amdgpu_waves_per_eu(Shape<T, MN, MC, MG, MP, 0, DR, LAY>::kWPE))) MG_VGPR_ATTR void k_env_step(
    const mg_model* __restrict__ m, const void* __restrict__ timg, mg_sim_params p, mg_task_params tp, mg_state_views v,
    mg_task_buffers tb, int n, mg_replay rp, unsigned* __restrict__ wq, MgOrder ord) {
  using SH = Shape<T, MN, MC, MG, MP, 0, DR, LAY>;
  constexpr int E = SH::E, W = SH::W;
  __shared__ mg::BankSlot<mg::TeamLDSOf<T, MN, MC, 0, MG, MP, LAY>, T> lds[E];
  __shared__ mg::ModelTile<MN, MG, MP> tile;
  __shared__ mg::DrTile<DR ? MN : 1, DR ? MG : 1> drt[DR ? E : 1];
  span_start(ord.clk, (int)blockIdx.x * W + (int)(threadIdx.x / 64));
  sort_totals_clear(ord);
  mg::copy_tile(&tile, static_cast<const mg::ModelTile<MN, MG, MP>*>(timg));
  __syncthreads();  // the only block-wide barrier: every later phase synchronises its own wave
  if constexpr (SH::kStatic) {
    // the static grid, one item per wave (one-wave blocks free their slot as soon as their wave is done)
    const int item = (int)blockIdx.x * W + (int)(threadIdx.x / 64);
    if (item * SH::E1 < n) env_step_item<T, MN, MC, MG, MP, DR, RP, TGS, LAY>(m, tile, lds, drt, p, tp, v, tb, n, rp, item, ord);
    span_end(ord.clk, item);
    order_done(ord, (int)gridDim.x * W);
  } else {
    // multi-wave blocks: the work queue (wq_next), the grid being the resident capacity
    const int nit = (n + SH::E1 - 1) / SH::E1, gwv = (int)gridDim.x * W;
    for (int item = (int)blockIdx.x * W + (int)(threadIdx.x / 64); item < nit; item = wq_next(wq, gwv)) {
      const int z = opaque_zero();
      env_step_item<T, MN, MC, MG, MP, DR, RP, TGS, LAY>(m + z, (&tile)[z], lds + z, drt + z, (&p)[z], (&tp)[z], (&v)[z], (&tb)[z], n,
                                               (&rp)[z], item, (&ord)[z]);
    }
    span_end(ord.clk, (int)blockIdx.x * W + (int)(threadIdx.x / 64));
    order_done(ord, gwv);
    wq_done(wq, gwv);
  }
}

// ------------------------------------------------------------------------------------------------ hand tasks
// index of DOF d in the actuated list (action column), -1 if not actuated
__device__ __forceinline__ int hand_action_of(const mg_task_params& tp, int d) {
  for (int i = 0; i < tp.num_actions; i++)
    if (tp.actuated_dof[i] == d) return i;
  return -1;
}

// The whole ShadowHand VecTask.step for one env, fused: pre_physics_step (masked goal / env resets,
// PD targets) -> simulate x substeps -> post_physics_step (full_state obs, reward, partial sums of
// the running mean) -> timeout, obs clamp, state write-back.  One team of T lanes per env.
// RP: physics-bypass replay instance (mg_env_step_replay), as k_env_step's.
// one work item of k_hand_step: the E1 teams of one wave (item = the wave's global index)
template <int T, int MN, int MC, int MG, int MP, int OT, bool DR, bool RP, bool TGS = false>
__device__ __forceinline__ void hand_step_item(
    const mg_model* __restrict__ m, const mg::ModelTile<MN, MG, MP, mg::tile_hull_verts(OT)>& tile, mg::BankSlot<mg::TeamLDSOf<T, MN, MC, OT, MG, MP, 0>, T>* lds,
    mg::DrTile<DR ? MN : 1, DR ? MG : 1>* drt, const mg_sim_params& p, const mg_task_params& tp, const mg_state_views& v,
    const mg_task_buffers& tb, int n, const mg_replay& rp, int item, const MgOrder& ord) {
  using SH = Shape<T, MN, MC, MG, MP, OT, DR>;
  const int team = threadIdx.x / T;
  const int slot = item * SH::E1 + (int)(threadIdx.x & 63) / T;
  const bool valid = slot < n;
  const int e = ordered_actor(ord, slot, n, 1);
  const int ec = valid ? e : n - 1;
  const int nd = m->num_dofs, ns = m->num_sensors, na = tp.num_actions, no = tp.num_obs;
  const int nb = m->num_bodies, nbe = nb + 2;
  mg::TeamLDSOf<T, MN, MC, OT, MG, MP, 0>& L = lds[team].v;
  mg::Team<T, MN, MC, MG, MP, OT, TGS> t;
  t.init(&L, &tile, m, &p, SH::W > 1);
  if constexpr (DR) {  // domain randomization: this actor's env_props row into the team's DrTile
    mg::load_dr<T>(&drt[team], v.env_props + (size_t)v.env_props_stride * ec, m, t.tl);
    t.drn = &drt[team].node[0][0];
    t.drg = drt[team].geom;
    t.drt = &drt[team].ten[0][0];
    t.dro = drt[team].obj;
  }
  t.ph_start();
  const uint64_t gid = (uint64_t)(tb.env_offset + ec);
  const bool env_reset = tb.reset[ec] != 0, goal_reset = tb.reset_goal[ec] != 0;
  float* root = v.root_states + (size_t)39 * ec;
  // ---- pre_physics_step: goal / object resets staged in LDS by the team leader
  if (t.tl == 0) {
    float* gr = L.goal;
    float* gs = L.goal + 13;
    if (env_reset || goal_reset) {
      const int c0 = env_reset ? 57 : 0;  // env reset: reset_idx's own reset_target_pose draw wins
      mg::h_reset_goal(tp, mg::h_rand_pm1(mg::h_uniform(tb, ec, gid, c0)),
                       mg::h_rand_pm1(mg::h_uniform(tb, ec, gid, c0 + 1)), gs, gr);
      for (int k = 7; k < 13; k++) gs[k] = tb.goal_states[(size_t)13 * ec + k];
    } else {
      for (int k = 0; k < 13; k++) { gr[k] = root[26 + k]; gs[k] = tb.goal_states[(size_t)13 * ec + k]; }
    }
    // random object forces: reset_idx zeroes / redraws the probability, pre_physics_step decays / draws
    float f[3] = {0.0f, 0.0f, 0.0f};
    if (v.rb_forces || tb.random_force_prob) {
      const float* fr = v.rb_forces ? v.rb_forces + ((size_t)nbe * ec + nb) * 3 : nullptr;
      if (fr)
        for (int k = 0; k < 3; k++) f[k] = fr[k];
      if (valid) mg::h_object_force(tp, tb, ec, gid, env_reset, f);
    }
    for (int k = 0; k < 3; k++) L.oforce[k] = f[k];
    L.oforce[3] = v.rb_force_space == MG_LOCAL_SPACE ? 1.0f : 0.0f;
    if (env_reset) {
      float r[5];
      for (int k = 0; k < 5; k++) r[k] = mg::h_rand_pm1(mg::h_uniform(tb, ec, gid, 4 + k));
      for (int k = 0; k < 3; k++) L.oroot[k] = tp.object_start[k] + tp.reset_position_noise * r[k];
      mg::h_object_reset_rotation(tp, r[3], r[4], L.oroot + 3);
      for (int k = 7; k < 13; k++) L.oroot[k] = 0.0f;
    } else {
      for (int k = 0; k < 13; k++) L.oroot[k] = root[13 + k];
    }
  }
  mg::wsync();
  t.load(root, v.dof_state + (size_t)2 * nd * ec, nullptr, L.oroot, nullptr);
  float prev = 0.0f;
  if (t.node > 0) {  // DOF lanes: reset_idx's DOF draw, then actions -> PD targets
    const int d = t.node - 1;
    float cur;
    if (env_reset) {
      const float rp = mg::h_rand_pm1(mg::h_uniform(tb, ec, gid, 9 + d));
      const float rv = mg::h_rand_pm1(mg::h_uniform(tb, ec, gid, 9 + nd + d));
      const float dmax = tp.dof_upper[d] - tp.initial_dof_pos[d], dmin = tp.dof_lower[d] - tp.initial_dof_pos[d];
      const float pos = tp.initial_dof_pos[d] + tp.reset_dof_pos_noise * (dmin + (dmax - dmin) * 0.5f * (rp + 1.0f));
      t.qj = pos;
      t.nu = 0.0f + tp.reset_dof_vel_noise * rv;
      prev = pos;
      cur = pos;
    } else {
      prev = tb.prev_targets[(size_t)nd * ec + d];
      cur = v.dof_targets[(size_t)nd * ec + d];
    }
    const int ai = hand_action_of(tp, d);
    if (ai >= 0) {
      const float a = mg::clampf(tb.actions[(size_t)na * ec + ai], tp.clip_actions);
      cur = mg::h_target(tp, d, a, prev);
      prev = cur;
    }
    t.tgt = cur;
  }
  // ---- gym.simulate
  t.ph_mark(14);
  if constexpr (RP) {  // replaced by the injected post-simulate state; the pre-physics state goes out
    if (valid && rp.pre_root_states) {
      float* pr = rp.pre_root_states + (size_t)39 * e;
      for (int k = t.tl; k < 13; k += T) { pr[k] = root[k]; pr[13 + k] = L.oroot[k]; pr[26 + k] = L.goal[k]; }
    }
    if (valid && rp.pre_dof_state && t.node > 0) {
      rp.pre_dof_state[(size_t)2 * nd * e + 2 * (t.node - 1)] = t.qj;
      rp.pre_dof_state[(size_t)2 * nd * e + 2 * (t.node - 1) + 1] = t.nu;
    }
    mg::wsync();
    for (int k = t.tl; k < 13; k += T) L.oroot[k] = rp.root_states[(size_t)39 * ec + 13 + k];
    for (int k = t.tl; k < 2 * nd; k += T) L.st().dof[k] = rp.dof_state[(size_t)2 * nd * ec + k];
    for (int k = t.tl; k < 6 * ns; k += T) L.st().sens[k] = rp.sensors ? rp.sensors[(size_t)6 * ns * ec + k] : 0.0f;
    for (int k = t.tl; k < nd; k += T) L.st().dforce[k] = rp.dof_force ? rp.dof_force[(size_t)nd * ec + k] : 0.0f;
  } else {
    // controlFrequencyInv: gym.simulate x cfi between one pre- and one post_physics_step (vec_task.py:381-384)
    const int nsub = p.substeps * (tp.control_freq_inv > 1 ? tp.control_freq_inv : 1);
    for (int st = 0; st < nsub; st++) t.substep();
    t.outputs(L.st().sens, L.st().dforce,
              (valid && v.net_contact_forces) ? v.net_contact_forces + (size_t)3 * nbe * e : nullptr);
    t.stage_state();
  }
  mg::wsync();
  t.ph_mark(8);
  // NaN guard: a non-finite hand / object state after the step -> reset = 1 (the next
  // step's pre_physics reset_idx restores the env), reward 0, zero observation row
  bool nf = false;
  for (int k = t.tl; k < 13; k += T) nf = nf || !isfinite(L.oroot[k]);
  for (int k = t.tl; k < 2 * nd; k += T) nf = nf || !isfinite(L.st().dof[k]);
  const bool bad = ((__ballot(nf) >> t.tb) & mg::team_bits<T>()) != 0ull;
  // ---- post_physics_step: full_state obs staged in LDS (team-parallel), reward on the leader
  const int64_t progress_in = env_reset ? 0 : tb.progress[ec];
  float* rbs = v.rigid_body_states + (size_t)13 * nbe * ec;
  // rigid-body states of the hand once (one lane per body) into the dead row storage: the fingertip
  // observations and the rigid_body_states write-back both read them
  float* bst = &L.rows()[0].b;
  if constexpr (RP) {
    for (int k = t.tl; k < 13 * nb; k += T) bst[k] = rp.rigid_body_states[(size_t)13 * nbe * ec + k];
  } else {
    for (int b = t.tl; b < nb; b += T) t.body_state(b, bst + 13 * b);
  }
  mg::wsync();
  {
    const float* gs = L.goal + 13;
    float qdiff[4];
    const float gc[4] = {-gs[3], -gs[4], -gs[5], gs[6]};
    mg::t_quat_mul(L.oroot + 3, gc, qdiff);
    for (int k = t.tl; k < no; k += T) {
      const int mk = tp.obs_map[k], seg = mk >> 8, i = mk & 255;   // column -> (segment, index)
      float x;
      if (seg == mg::HS_ACTIONS) {  // self.actions (clamped)
        x = mg::clampf(tb.actions[(size_t)na * ec + i], tp.clip_actions);
      } else if (seg == mg::HS_FT_STATE || seg == mg::HS_FT_POS) {  // fingertip state from the post-step FK
        int b, c;
        mg::h_ft_ref(tp, seg, i, &b, &c);
        x = bst[13 * b + c];
      } else {
        x = mg::h_obs_value(tp, seg, i, L.st().dof, L.st().dforce, L.oroot, gs, qdiff, L.st().sens, nullptr);
      }
      L.obs[k] = x;
    }
  }
  mg::wsync();
  int64_t ro = 0;
  float fin = 0.0f;
  if (t.tl == 0) {
    const float* gs = L.goal + 13;
    float succ = env_reset ? 0.0f : tb.successes[ec], rew;
    int64_t prog = progress_in + 1, go;
    mg::h_reward(tp, L.oroot, L.oroot + 3, gs, gs + 3, L.obs + (no - na), 0, 0, &prog, &succ, &rew, &ro, &go);
    if (bad) {
      ro = 1;
      rew = 0.0f;
    }
    if (valid) {
      tb.rew[e] = rew;
      tb.reset[e] = ro;
      tb.reset_goal[e] = go;
      tb.progress[e] = prog;
      tb.successes[e] = succ;
      tb.timeout[e] = (uint8_t)((prog >= (int64_t)tp.max_episode_length - 1) && (ro != 0));
      // a guard-forced reset counts as a reset of the running mean, with no successes (its succ comes
      // from a non-finite state)
      fin = bad ? 0.0f : succ * (float)ro;
      if (tb.out_pack) {
        tb.out_pack[(size_t)(no + 2) * e + no] = rew;
        tb.out_pack[(size_t)(no + 2) * e + no + 1] = (float)ro;
      }
    } else {
      ro = 0;
    }
  }
  // partial sums of the global running mean: wave reduce, one atomic pair per wave
  unsigned long long cr = (unsigned long long)ro, cf = (unsigned long long)fin;
  for (int off = 32; off >= 1; off >>= 1) {
    cr += __shfl_xor(cr, off);
    cf += __shfl_xor(cf, off);
  }
  if ((threadIdx.x & 63) == 0 && (cr | cf)) {
    atomicAdd((unsigned long long*)&tb.reduce_scratch[0], cr);
    atomicAdd((unsigned long long*)&tb.reduce_scratch[1], cf);
  }
  if (valid) {  // write-back (gym layouts), team-cooperative
    float* o = tb.obs + (size_t)no * e;
    for (int k = t.tl; k < no; k += T) {
      const float x = bad ? 0.0f : L.obs[k];
      o[k] = x;
      if (tb.obs_clamped) tb.obs_clamped[(size_t)no * e + k] = mg::clampf(x, tp.clip_obs);
    }
    if (tb.out_pack) {  // the gather's message row [clamped obs | rew | reset] (migym/dist.py)
      float* pk = tb.out_pack + (size_t)(no + 2) * e;
      for (int k = t.tl; k < no; k += T) pk[k] = bad ? 0.0f : mg::clampf(L.obs[k], tp.clip_obs);
    }
    if (tb.actions_out)
      for (int k = t.tl; k < na; k += T) tb.actions_out[(size_t)na * e + k] = L.obs[no - na + k];
    for (int k = t.tl; k < 13; k += T) {
      root[13 + k] = L.oroot[k];
      root[26 + k] = L.goal[k];
      tb.goal_states[(size_t)13 * e + k] = L.goal[13 + k];
    }
    for (int k = t.tl; k < 2 * nd; k += T) v.dof_state[(size_t)2 * nd * e + k] = L.st().dof[k];
    if (t.node > 0) {
      const int d = t.node - 1;
      const_cast<float*>(v.dof_targets)[(size_t)nd * e + d] = t.tgt;
      tb.prev_targets[(size_t)nd * e + d] = prev;
    }
    if (v.sensors)
      for (int k = t.tl; k < 6 * ns; k += T) v.sensors[(size_t)6 * ns * e + k] = L.st().sens[k];
    if (v.dof_force)
      for (int k = t.tl; k < nd; k += T) v.dof_force[(size_t)nd * e + k] = L.st().dforce[k];
    for (int k = t.tl; k < 13 * nb; k += T) rbs[k] = bst[k];
    for (int k = t.tl; k < 26; k += T) rbs[13 * nb + k] = k < 13 ? L.oroot[k] : L.goal[k - 13];
    if (v.rb_forces && t.tl < 3) v.rb_forces[((size_t)nbe * e + nb) * 3 + t.tl] = L.oforce[t.tl];
    if (tb.states) {  // asymmetric_observations: the full_state layout (compute_full_state(asymm_obs=True))
      const float* gs = L.goal + 13;
      float qdiff[4];
      const float gc[4] = {-gs[3], -gs[4], -gs[5], gs[6]};
      mg::t_quat_mul(L.oroot + 3, gc, qdiff);
      for (int k = t.tl; k < tp.num_states; k += T) {
        const int mk = tp.state_map[k], seg = mk >> 8, i = mk & 255;
        float x;
        if (seg == mg::HS_FT_STATE || seg == mg::HS_FT_POS) {
          int b, c;
          mg::h_ft_ref(tp, seg, i, &b, &c);
          x = bst[13 * b + c];
        } else {
          x = mg::h_obs_value(tp, seg, i, L.st().dof, L.st().dforce, L.oroot, gs, qdiff, L.st().sens,
                              L.obs + (no - na));
        }
        tb.states[(size_t)tp.num_states * e + k] = bad ? 0.0f : x;   // NaN guard, as for obs
      }
    }
  }
  if (valid && t.tl == 0) {  // the next launch's order
    if (ord.wcnt) order_append(ord, L.nrows, e);
    else if (ord.cost) ord.cost[e] = (unsigned char)(L.nrows < 255 ? L.nrows : 255);
  }
  t.ph_mark(9);
  MG_PHASE_FLUSH(t, item)
}

template <int T, int MN, int MC, int MG, int MP, int OT, bool DR, bool RP, bool TGS = false>
__global__ __launch_bounds__((Shape<T, MN, MC, MG, MP, OT, DR>::kThreads)) __attribute__((amdgpu_waves_per_eu(Shape<T, MN, MC, MG, MP, OT, DR>::kWPE))) void k_hand_step(
    const mg_model* __restrict__ m, const void* __restrict__ timg, mg_sim_params p, mg_task_params tp, mg_state_views v,
    mg_task_buffers tb, int n, mg_replay rp, unsigned* __restrict__ wq, MgOrder ord) {
  using SH = Shape<T, MN, MC, MG, MP, OT, DR>;
  constexpr int E = SH::E, W = SH::W;
  __shared__ mg::BankSlot<mg::TeamLDSOf<T, MN, MC, OT, MG, MP, 0>, T> lds[E];
  __shared__ mg::ModelTile<MN, MG, MP, mg::tile_hull_verts(OT)> tile;
  __shared__ mg::DrTile<DR ? MN : 1, DR ? MG : 1> drt[DR ? E : 1];
  span_start(ord.clk, (int)blockIdx.x * W + (int)(threadIdx.x / 64));
  sort_totals_clear(ord);
  mg::copy_tile(&tile, static_cast<const mg::ModelTile<MN, MG, MP, mg::tile_hull_verts(OT)>*>(timg));
  __syncthreads();  // the only block-wide barrier: every later phase synchronises its own wave
  if constexpr (W == 1) {  // as k_env_step
    if ((int)blockIdx.x * SH::E1 < n) hand_step_item<T, MN, MC, MG, MP, OT, DR, RP, TGS>(m, tile, lds, drt, p, tp, v, tb, n, rp, blockIdx.x, ord);
    span_end(ord.clk, (int)blockIdx.x * W + (int)(threadIdx.x / 64));
    order_done(ord, (int)gridDim.x);
  } else {
    const int nit = (n + SH::E1 - 1) / SH::E1, gwv = (int)gridDim.x * W;
    for (int item = (int)blockIdx.x * W + (int)(threadIdx.x / 64); item < nit; item = wq_next(wq, gwv)) {
      const int z = opaque_zero();
      hand_step_item<T, MN, MC, MG, MP, OT, DR, RP, TGS>(m + z, (&tile)[z], lds + z, drt + z, (&p)[z], (&tp)[z], (&v)[z],
                                                    (&tb)[z], n, (&rp)[z], item, (&ord)[z]);
    }
    span_end(ord.clk, (int)blockIdx.x * W + (int)(threadIdx.x / 64));
    order_done(ord, gwv);
    wq_done(wq, gwv);
  }
}

// launch helper: grid of ceil(n / teams-per-block) blocks of the instance's shape
template <class SH, class K, class... A>
static void launch(K kern, hipStream_t s, int n, A... args) {
  hipLaunchKernelGGL(kern, dim3((n + SH::E - 1) / SH::E), dim3(SH::kThreads), 0, s, args...);
}

// launch of a step kernel: multi-wave blocks get min(blocks of the whole batch, resident blocks) blocks (the
// work queue; occupancy query cached per kernel and device), one-wave blocks one block per item
template <class SH, class K, class... A>
static int launch_wq(K kern, hipStream_t s, const mg_sim* sim, bool ordered, A... args) {
  struct Entry { const void* k; int dev, blocks; };
  static Entry cache[32];  // (kernel, device) -> resident blocks
  const void* kp = reinterpret_cast<const void*>(kern);
  int resident = 0;
  for (const Entry& c : cache)
    if (c.k == kp && c.dev == sim->device) resident = c.blocks;
  if (resident <= 0) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kp, SH::kThreads, MG_LDS_PAD + sim->lds_pad) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, sim->device) != hipSuccess || per_cu <= 0 ||
        cus <= 0)
      return fail(MG_EDEVICE, "mg_env_step: occupancy query failed");
    resident = per_cu * cus;
    if (getenv("MIGYM_PRINT_OCC"))  // diagnostics: the resident blocks the runtime reports for this kernel
      fprintf(stderr, "migym: step kernel W=%d: %d blocks per CU (%d waves), lds pad %d\n", SH::W, per_cu,
              per_cu * SH::W, MG_LDS_PAD + sim->lds_pad);
    for (Entry& c : cache)
      if (!c.k) { c = Entry{kp, sim->device, resident}; break; }
  }
  const int items = (sim->n + SH::E1 - 1) / SH::E1;
  const int need = (items + SH::W - 1) / SH::W;
  const int blocks = SH::kStatic ? need : (need < resident ? need : resident);
  unsigned long long* clk = nullptr;  // mg_kernel_span_begin: this launch's slot, one (start, end) pair per wave
  if (sim->d_span && sim->span_next < sim->span_cap && blocks * SH::W <= sim->span_stride) {
    mg_sim* ms = const_cast<mg_sim*>(sim);   // recording bookkeeping only
    clk = ms->d_span + 2 * (size_t)ms->span_stride * ms->span_next;
    ms->span_waves[ms->span_next++] = blocks * SH::W;
  }
  MgOrder ord{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, sim->bq_cap, clk, nullptr,
              sim->order_unit};
  if (ordered && sim->order_mode == kOrderSort) {
    ord.order = sim->order_valid ? sim->d_order : nullptr;
    ord.cost = sim->d_cost;
    ord.tot_clear = sim->d_osort;
  } else if (ordered && sim->order_mode == kOrderLists) {
    const int rs = (int)(sim->order_steps & 1), ws = 1 - rs;   // this launch reads set rs, writes set ws
    ord.rcnt = sim->order_valid ? sim->d_bq + rs * kOrderBuckets : nullptr;
    ord.rlist = sim->d_blist + (size_t)rs * kOrderBuckets * sim->bq_cap;
    ord.wcnt = sim->d_bq + ws * kOrderBuckets;
    ord.wlist = sim->d_blist + (size_t)ws * kOrderBuckets * sim->bq_cap;
    ord.rclear = sim->d_bq + rs * kOrderBuckets;
    ord.done = sim->d_bq + 2 * kOrderBuckets;
  }
  // one-wave blocks: the static grid, one block per item; multi-wave blocks: the resident capacity (work queue)
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(SH::kThreads), MG_LDS_PAD + sim->lds_pad, s, args..., sim->d_wq, ord);
  return MG_OK;
}

template <int T, int MN, int MC, int MG, int MP, int OBJ, int LAY>
int BuildTile<T, MN, MC, MG, MP, OBJ, LAY>::run(mg_sim* sim) {
  using MT = mg::ModelTile<MN, MG, MP, mg::tile_hull_verts(OBJ)>;   // the kernels' tile type (Team::MT)
  MT* img = new (std::nothrow) MT();
  if (!img) return fail(MG_ENOMEM, "mg_sim_create: out of host memory (model tile)");
  mg::build_tile(img, &sim->host_model);
  int rc = MG_OK;
  if (hipMalloc(&sim->d_tile, sizeof(MT)) != hipSuccess) {
    sim->d_tile = nullptr;
    rc = fail(MG_ENOMEM, "mg_sim_create: hipMalloc(model tile) failed");
  } else if (hipMemcpy(sim->d_tile, img, sizeof(MT), hipMemcpyHostToDevice) != hipSuccess) {
    rc = fail(MG_EDEVICE, "mg_sim_create: model tile upload failed");
  }
  delete img;
  return rc;
}

template <int T, int MN, int MC, int MG, int MP, int OBJ, int LAY>
int RunSimulate<T, MN, MC, MG, MP, OBJ, LAY>::run(hipStream_t s, const mg_sim* sim) {
  if (!sim->d_tile) return fail(MG_ECAPACITY, "mg_sim_simulate: no model tile (model exceeds every kernel instance)");
  // the domain-randomized instance reads each actor's env_props row (mg_dr_apply); TGS runs its own instances
  const bool tgs = sim->params.solver_type == MG_SOLVER_TGS;
  if (sim->views.env_props) {
    if (tgs)
      launch<Shape<T, MN, MC, MG, MP, OBJ, true, LAY>>(k_simulate<T, MN, MC, MG, MP, OBJ, true, true, LAY>, s, sim->n, sim->d_model,
                                                   (const void*)sim->d_tile, sim->params, sim->views, sim->n);
    else
      launch<Shape<T, MN, MC, MG, MP, OBJ, true, LAY>>(k_simulate<T, MN, MC, MG, MP, OBJ, true, false, LAY>, s, sim->n, sim->d_model,
                                                   (const void*)sim->d_tile, sim->params, sim->views, sim->n);
  } else if (tgs) {
    launch<Shape<T, MN, MC, MG, MP, OBJ, false, LAY>>(k_simulate<T, MN, MC, MG, MP, OBJ, false, true, LAY>, s, sim->n, sim->d_model,
                                                  (const void*)sim->d_tile, sim->params, sim->views, sim->n);
  } else {
    launch<Shape<T, MN, MC, MG, MP, OBJ, false, LAY>>(k_simulate<T, MN, MC, MG, MP, OBJ, false, false, LAY>, s, sim->n, sim->d_model,
                                                  (const void*)sim->d_tile, sim->params, sim->views, sim->n);
  }
  return MG_OK;
}

template <int T, int MN, int MC, int MG, int MP, int OBJ, int LAY>
int RunEnvStep<T, MN, MC, MG, MP, OBJ, LAY>::run(hipStream_t s, const mg_sim* sim, const mg_task_params* tp,
                                                  const mg_task_buffers* tb, const mg_replay* rp) {
  using TL = mg::TeamLDSOf<T, MN, MC, OBJ, MG, MP, LAY>;
  if (!sim->d_tile) return fail(MG_ECAPACITY, "mg_env_step: no model tile (model exceeds every kernel instance)");
  // observations are staged in the (dead) row storage of the team's LDS before the coalesced store
  if (!OBJ && (size_t)tp->num_obs * sizeof(float) > TL::kObsStageBytes)
    return fail(MG_ECAPACITY, "mg_env_step: observation row exceeds the kernel's staging area");
  // hand tasks stage the rigid-body states of the articulation in the same storage, the observation
  // row in the contact storage; the observation / states column maps hold 256 entries
  if (OBJ && (size_t)13 * sim->host_model.num_bodies * sizeof(float) > TL::kObsStageBytes)
    return fail(MG_ECAPACITY, "mg_env_step: rigid bodies exceed the kernel's staging area");
  if (OBJ && (tp->num_obs < 0 || (size_t)tp->num_obs > sizeof(TL::obs) / sizeof(float)))
    return fail(MG_ECAPACITY, "mg_env_step: observation row exceeds the hand kernel's staging area");
  if (OBJ && (tp->num_states < 0 || tp->num_states > (int)(sizeof(tp->state_map) / sizeof(tp->state_map[0]))))
    return fail(MG_ECAPACITY, "mg_env_step: num_states exceeds the hand kernel's states map");
  if (rp && sim->views.env_props)
    return fail(MG_EINVAL, "mg_env_step_replay: no replay instance with domain randomization");
  const mg_replay r = rp ? *rp : mg_replay{};
  const void* ti = sim->d_tile;
  const bool tgs = sim->params.solver_type == MG_SOLVER_TGS;  // TGS runs its own instances (not the replay's: no physics)
  if constexpr (OBJ != 0) {
    mg_task_params tpm = *tp;  // observation column maps (hand_task.hpp h_fill_maps)
    mg::h_fill_maps(&tpm);
    if (rp)
      return launch_wq<Shape<T, MN, MC, MG, MP, OBJ, false>>(k_hand_step<T, MN, MC, MG, MP, OBJ, false, true>, s, sim, false,
                                                    sim->d_model, ti, sim->params, tpm, sim->views, *tb, sim->n, r);
    else if (sim->views.env_props && tgs)
      return launch_wq<Shape<T, MN, MC, MG, MP, OBJ, true>>(k_hand_step<T, MN, MC, MG, MP, OBJ, true, false, true>, s, sim,
                                                   true, sim->d_model, ti, sim->params, tpm, sim->views, *tb, sim->n, r);
    else if (sim->views.env_props)
      return launch_wq<Shape<T, MN, MC, MG, MP, OBJ, true>>(k_hand_step<T, MN, MC, MG, MP, OBJ, true, false>, s, sim, true,
                                                   sim->d_model, ti, sim->params, tpm, sim->views, *tb, sim->n, r);
    else if (tgs)
      return launch_wq<Shape<T, MN, MC, MG, MP, OBJ, false>>(k_hand_step<T, MN, MC, MG, MP, OBJ, false, false, true>, s, sim,
                                                    true, sim->d_model, ti, sim->params, tpm, sim->views, *tb, sim->n, r);
    else
      return launch_wq<Shape<T, MN, MC, MG, MP, OBJ, false>>(k_hand_step<T, MN, MC, MG, MP, OBJ, false, false>, s, sim, true,
                                                    sim->d_model, ti, sim->params, tpm, sim->views, *tb, sim->n, r);
  } else {
    if (rp)
      return launch_wq<Shape<T, MN, MC, MG, MP, 0, false, LAY>>(k_env_step<T, MN, MC, MG, MP, false, true, false, LAY>, s, sim, false, sim->d_model,
                                                  ti, sim->params, *tp, sim->views, *tb, sim->n, r);
    else if (sim->views.env_props && tgs)
      return launch_wq<Shape<T, MN, MC, MG, MP, 0, true, LAY>>(k_env_step<T, MN, MC, MG, MP, true, false, true, LAY>, s, sim, true,
                                                 sim->d_model, ti, sim->params, *tp, sim->views, *tb, sim->n, r);
    else if (sim->views.env_props)
      return launch_wq<Shape<T, MN, MC, MG, MP, 0, true, LAY>>(k_env_step<T, MN, MC, MG, MP, true, false, false, LAY>, s, sim, true, sim->d_model,
                                                 ti, sim->params, *tp, sim->views, *tb, sim->n, r);
    else if (tgs)
      return launch_wq<Shape<T, MN, MC, MG, MP, 0, false, LAY>>(k_env_step<T, MN, MC, MG, MP, false, false, true, LAY>, s, sim, true,
                                                  sim->d_model, ti, sim->params, *tp, sim->views, *tb, sim->n, r);
    else
      return launch_wq<Shape<T, MN, MC, MG, MP, 0, false, LAY>>(k_env_step<T, MN, MC, MG, MP, false, false, false, LAY>, s, sim, true, sim->d_model,
                                                  ti, sim->params, *tp, sim->views, *tb, sim->n, r);
  }
  return MG_OK;
}

template <int I>
int phase_buf_publish(unsigned long long* buf) {
#ifdef MG_PHASE_TIMING
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_phase_buf), &buf, sizeof(buf)) != hipSuccess)
    return fail(MG_EDEVICE, "mg_debug_phase_cycles: buffer publish failed");
  return MG_OK;
#else
  (void)buf;
  return fail(MG_EINVAL, "mg_debug_phase_cycles: library built without MG_PHASE_TIMING");
#endif
}
}  // namespace mgi
