/*
 * oracle.h — CPU restatement used ONLY as the parity checker and the CPU
 * baseline (tests/, __graft_entry__.smoke(), bench.py cpu_baseline leg).
 * Nothing in the product links or calls this library.
 *
 * PARITY STATUS
 *   obs / reward / reset bookkeeping: PINNED.  The restatement follows the
 *     reference's @torch.jit.script functions (tasks/ant.py:325-408,
 *     tasks/humanoid.py:323-413, tasks/cartpole.py:119-196,
 *     utils/torch_jit_utils.py:41-276) and VecTask.step ordering
 *     (tasks/base/vec_task.py:362-410); tests/test_oracle_golden.py checks it
 *     against tests/golden/jit_*.npz and trace_*.npz, produced by running the
 *     reference code itself (tests/golden/make_golden.py, make_traces.py).
 *   physics (gym.simulate): PARITY UNPINNED.  The reference physics is the
 *     closed isaacgym/PhysX binary (not in the reference tree, not installable
 *     offline).  This file restates the build's own documented algorithm
 *     (DESIGN.md §Physics): composite-rigid-body mass matrix + Cholesky in
 *     fp64 — deliberately NOT the O(n) articulated-body recursion the HIP
 *     kernels use — with the same contact set, PGS row order and integrator,
 *     and is pinned by analytic known-answer tests (free fall, energy,
 *     pendulum, joint limits, resting contact) in tests/test_oracle_physics.py.
 */
#ifndef MIGYM_ORACLE_H
#define MIGYM_ORACLE_H
#include "../include/migym.h"

#ifdef __cplusplus
extern "C" {
#endif

/* counter-based uniform in [0,1): identical integer recipe on the GPU */
float orc_uniform(uint64_t seed, uint64_t env, uint64_t counter, uint32_t k);

/* gym.simulate on host buffers (gym layouts), fp64 internally, one actor per
 * row; `threads` OpenMP threads (0 = library default). */
int orc_simulate(const mg_model* m, const mg_sim_params* p, int32_t n, float* root_states, float* dof_state,
                 const float* dof_actuation, float* sensors, float* dof_force, int32_t threads);

/* gym.simulate on the full state views: object/goal root rows, PD targets and rigid-body states
 * of hand tasks included (views->dof_targets may be NULL = zero targets). */
int orc_simulate_views(const mg_model* m, const mg_sim_params* p, int32_t n, const mg_state_views* v,
                       int32_t threads);

/* Debug/KAT hooks for one actor: mass matrix (nv*nv row-major, includes the
 * armature + implicit damping/stiffness diagonal for substep h) and the
 * unconstrained generalized acceleration. */
int orc_mass_matrix(const mg_model* m, const mg_sim_params* p, const float* root13, const float* dof2,
                    double* M_out);
int orc_free_acceleration(const mg_model* m, const mg_sim_params* p, const float* root13, const float* dof2,
                          const float* tau, double* qacc_out);
/* contacts detected for one actor at the given state: returns count; writes
 * (node, px,py,pz, nx,ny,nz, depth, nodeB) records of 9 doubles */
int orc_contacts(const mg_model* m, const mg_sim_params* p, const float* root13, const float* dof2, double* out,
                 int32_t cap);
/* egg narrowphase KAT hook (GJK + shrunk-core retry): kind 0 segment p0,p1 / kind 1 box c, R (row-major),
 * h, plus radius, vs the origin-centred ellipsoid e; out = point(3), normal(3), distance */
int orc_ellipsoid_contact(int32_t kind, const double* shape, double radius, const double* e, double* out);
/* edge-edge KAT hook: hand box c (3), R row-major (9), h (3) in the object box's frame (half extents hb);
 * out = point(3), normal(3), separation; returns 1 when generated */
int orc_box_box_edge(const double* shape, const double* hb, double off, double* out);
/* the convex-mesh geom's plane distance of n geom-frame points: out = (distance, face) per point */
int orc_hull_distance(const mg_model* m, const double* pl, int32_t n, double* out);
int orc_hull_core_contact(const mg_model* m, const double* shape, double rB, double off, double* out);
/* parity-test support: bit mask of the physics discontinuities env e's gym.simulate passes near (delta m / rad
 * of a contact / pair / limit threshold with the row in use; drives within df of saturation; seg_box_sat ties) */
int orc_step_flips(const mg_model* m, const mg_sim_params* p, const mg_state_views* v, int32_t e, double delta,
                   double df);
/* world poses of the gym rigid bodies (n_bodies x 13, velocity at body COM) */
int orc_rigid_body_states(const mg_model* m, const float* root13, const float* dof2, float* out);

int orc_compute_observations(const mg_task_params* tp, int32_t n, const float* root_states, const float* dof_state,
                             const float* dof_force, const float* sensors, const float* actions,
                             float* potentials, float* prev_potentials, float* up_vec, float* heading_vec,
                             float* obs);
int orc_compute_reward(const mg_task_params* tp, int32_t n, const float* obs, const float* actions,
                       const float* potentials, const float* prev_potentials, const int64_t* progress,
                       int64_t* reset, float* rew);
int orc_post_physics(const mg_task_params* tp, const mg_state_views* v, const mg_task_buffers* tb, int32_t n);
int orc_reset_idx(const mg_task_params* tp, const mg_state_views* v, const mg_task_buffers* tb, const int32_t* ids,
                  int32_t n_ids, int32_t n);
int orc_env_step(const mg_model* m, const mg_sim_params* p, const mg_task_params* tp, const mg_state_views* v,
                 const mg_task_buffers* tb, int32_t n, int32_t threads);

/* in-hand manipulation task layer (oracle_hand.c): ShadowHand full_state */
void orc_randomize_rotation(float r0, float r1, float* q);
int orc_hand_reward(const mg_task_params* tp, int32_t n, float max_episode_length, const float* object_pos,
                    const float* object_rot, const float* target_pos, const float* target_rot, const float* actions,
                    int64_t* reset, int64_t* reset_goal, int64_t* progress, float* successes, float* cons,
                    float* rew);
int orc_hand_pre_physics(const mg_model* m, const mg_task_params* tp, const mg_state_views* v,
                         const mg_task_buffers* tb, int32_t n);
int orc_hand_post_physics(const mg_model* m, const mg_task_params* tp, const mg_state_views* v,
                          const mg_task_buffers* tb, int32_t n);
int orc_hand_finalize(const mg_task_params* tp, const mg_task_buffers* tb);
int orc_hand_env_step(const mg_model* m, const mg_sim_params* p, const mg_task_params* tp,
                      const mg_state_views* v, const mg_task_buffers* tb, int32_t n, int32_t threads);

/* domain randomization (oracle_dr.c): restatements of mg_dr_apply / mg_dr_noise on host buffers */
int orc_dr_apply(const mg_dr_apply_args* a);
int orc_dr_noise(const mg_dr_noise_args* a);

#ifdef __cplusplus
}
#endif
#endif
