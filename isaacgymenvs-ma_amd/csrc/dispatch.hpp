// dispatch.hpp — the kernel instances (one per model capacity) and the host entry points each
// instance translation unit exports.  migym.hip sees only these declarations; inst.hip compiles
// one instance per translation unit (build.py runs them in parallel) from step_kernels.hpp.
#pragma once
#include "common.hpp"

// Kernel instances by capacity: team size T (>= velocity columns, nodes and sensors), nodes MN,
// contacts MC, geoms MG, self pairs MP, OBJ = the free object's type in hand-task envs (0: none; one
// instance per object shape, so the block's kernel carries no egg / pen code).  The smallest
// instance that fits the model is launched.
// (occupancy experiments only: the 16-lane locomotion instance's contact capacity)
#ifndef MG_ANT_MC
#define MG_ANT_MC 16
#endif
// LAY (last field): the team layout.  1 = the compact layout at three waves per SIMD (TeamLDSC), taken for batches of
// more than kCompactMinWaves waves; 0 = the classic layout at two waves per SIMD (TeamLDS) otherwise.  Twelve waves per
// CU pay where the batch fills several rounds of them; a batch that fits one or two rounds of the classic kernel's
// eight runs faster on it (Ant 16,384 envs = 4,096 waves: classic 139.4 vs compact 135.7 M env-steps/s; 8,192 envs:
// 128.6 vs 119.2 M; 32,768: 152.7 vs 176.8 M), so the two compact-capable capacities come in both layouts,
// compact first.
#define MG_INSTANCES(X)                                                                                                \
  X(8, 4, 8, 4, 0, 0, 0) X(16, 9, MG_ANT_MC, 16, 0, 0, 1) X(16, 9, MG_ANT_MC, 16, 0, 0, 0) X(16, 16, 24, 24, 32, 0, 0)   \
  X(32, 24, 32, 24, 160, 0, 1) X(32, 24, 32, 24, 160, 0, 0) X(32, 32, 48, 48, 192, 0, 0) X(64, 40, 48, 48, 192, 0, 0)    \
  X(32, 25, 24, 24, 24, MG_GT_BOX, 0) X(32, 25, 24, 24, 24, MG_GT_CAPSULE, 0) X(32, 25, 24, 24, 24, MG_GT_ELLIPSOID, 0)
#define MG_NUM_INST 11

namespace mgi {
struct InstDesc {
  int T, MN, MC, MG, MP, OBJ, LAY;
};
#define MG_DESC(T, MN, MC, MG, MP, OBJ, LAY) InstDesc{T, MN, MC, MG, MP, OBJ, LAY},
constexpr InstDesc kInst[] = {MG_INSTANCES(MG_DESC)};
#undef MG_DESC
static_assert(sizeof(kInst) / sizeof(kInst[0]) == MG_NUM_INST, "MG_NUM_INST must count MG_INSTANCES");

// the model tile image of an instance, built on the host and uploaded to sim->d_tile (mg_sim_create)
template <int T, int MN, int MC, int MG, int MP, int OBJ, int LAY>
struct BuildTile {
  static int run(mg_sim* sim);
};
// gym.simulate alone (k_simulate)
template <int T, int MN, int MC, int MG, int MP, int OBJ, int LAY>
struct RunSimulate {
  static int run(hipStream_t s, const mg_sim* sim);
};
// the whole VecTask.step (k_env_step / k_hand_step); rp != nullptr: physics-bypass replay instance
template <int T, int MN, int MC, int MG, int MP, int OBJ, int LAY>
struct RunEnvStep {
  static int run(hipStream_t s, const mg_sim* sim, const mg_task_params* tp, const mg_task_buffers* tb,
                 const mg_replay* rp);
};
// phase-timing build: publish the per-wave accumulator buffer to instance I's code object
template <int I>
int phase_buf_publish(unsigned long long* buf);

// the most tree nodes at one depth (the compact layout's ABA slots hold kCompactLevelSlots)
inline int level_width(const mg_model& m) {
  int depth[MG_MAX_NODES] = {0}, cnt[MG_MAX_NODES + 1] = {0}, w = 0;
  for (int i = 1; i < m.num_nodes && i < MG_MAX_NODES; i++) {
    depth[i] = (m.parent[i] >= 0 && m.parent[i] < i) ? depth[m.parent[i]] + 1 : 1;
    const int c = ++cnt[depth[i]];
    w = c > w ? c : w;
  }
  return w;
}
inline int model_lanes(const mg_model& m) {
  const int nv = (m.fixed_base ? 0 : 6) + m.num_dofs + (m.obj_type ? 6 : 0);
  return nv > m.num_sensors ? nv : m.num_sensors;
}
// the compact layout for batches of more than this many waves (64 / T actors each): the classic layout's resident
// capacity (256 CUs x 8 waves); a batch the classic kernel holds at once gains nothing from a third wave per SIMD
// and pays the compact layout's recomputation (round 6, same box, M env-steps/s classic / compact: Humanoid 4,096
// 21.3 / 17.8, Ant 8,192 121.5 / 118.8, MA-Ant 2,048 29.2 / 28.6; Ant 16,384 133.9 / 136.2, Humanoid 16,384
// 35.0 / 38.5)
constexpr long kCompactMinWaves = 2048;
inline bool layout_fits(int LAY, int T, int MN, int OBJ, const mg_model& m, long n_actors) {
  if (!LAY) return true;
  return mg_compact_layout(T, MN, OBJ) && level_width(m) <= kCompactLevelSlots &&
         (n_actors + 64 / T - 1) / (64 / T) > kCompactMinWaves;
}
#define MG_FITS(T, MN, MC, MG, MP, OBJ)                                                              \
  (m.num_nodes <= MN && max_contacts <= MC && model_lanes(m) <= T && (m.fixed_base || T >= 6) &&   \
   m.num_geoms <= MG && m.num_pairs <= MP && m.obj_type == (int)(OBJ))

// team size the dispatcher picks for a model (0: none fits)
inline int team_size(const mg_model& m, int max_contacts) {
#define MG_T(T, MN, MC, MG, MP, OBJ, LAY) \
  if (MG_FITS(T, MN, MC, MG, MP, OBJ)) return T;
  MG_INSTANCES(MG_T)
#undef MG_T
  return 0;
}

// the first instance that fits the model, its contact capacity and (for the layout) the batch of n_actors
template <template <int, int, int, int, int, int, int> class F, typename... A>
int dispatch(const mg_model& m, int max_contacts, long n_actors, A... args) {
#define MG_TRY(T, MN, MC, MG, MP, OBJ, LAY)                                                     \
  if (MG_FITS(T, MN, MC, MG, MP, OBJ) && layout_fits(LAY, T, MN, OBJ, m, n_actors)) {         \
    return F<T, MN, MC, MG, MP, OBJ, LAY>::run(args...);                                        \
  }
  MG_INSTANCES(MG_TRY)
#undef MG_TRY
  return fail(MG_ECAPACITY, "model exceeds the largest kernel instance");
}

// dispatch functor: the picked instance's team lanes and layout (mg_sim_kernel_layout)
template <int T, int MN, int MC, int MG, int MP, int OBJ, int LAY>
struct InstanceOf {
  static int run(int32_t* t, int32_t* lay) {
    *t = T;
    *lay = LAY;
    return 0;
  }
};
}  // namespace mgi
