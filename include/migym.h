/*
 * migym.h — C ABI of the MI355X-native physics-step + observation/reward path.
 *
 * This is the drop-in boundary that sits where the reference calls the closed
 * isaacgym tensor API.  Every entry point replaces one call
 * the reference's task layer makes on its hot path; the replaced call is cited
 * (paths relative to the reference checkout):
 *
 *   mg_sim_create        gym.create_sim + load_asset + create_env/create_actor loop
 *                        + prepare_sim              (tasks/base/vec_task.py:255-263,
 *                                                    tasks/ant.py:135-197)
 *   mg_sim_bind          gym.acquire_*_tensor + gymtorch.wrap_tensor
 *                                                   (tasks/ant.py:78-95, humanoid.py:75-95)
 *   mg_sim_simulate      gym.simulate(sim)          (tasks/base/vec_task.py:381-384)
 *   mg_set_indexed       gym.set_actor_root_state_tensor_indexed /
 *                        gym.set_dof_state_tensor_indexed
 *                                                   (tasks/ant.py:265-271, cartpole.py:153-155)
 *   mg_compute_observations   compute_{ant,humanoid}_observations / cartpole obs
 *                                                   (tasks/ant.py:374-408, humanoid.py:378-413,
 *                                                    cartpole.py:131-142)
 *   mg_compute_reward    compute_{ant,humanoid,cartpole}_reward
 *                                                   (tasks/ant.py:325-371, humanoid.py:323-375,
 *                                                    cartpole.py:180-196)
 *   (ShadowHand) mg_env_step also covers pre_physics_step's masked goal/env resets and
 *                        PD targets (shadow_hand.py:586-698) and compute_hand_reward's
 *                        global running mean (746-800, one finishing kernel).
 *   mg_env_step          one whole VecTask.step after the action tensor is on device:
 *                        clamp -> pre_physics_step -> simulate x controlFrequencyInv ->
 *                        post_physics_step (progress, masked reset_idx, obs, reward)
 *                        -> timeout_buf -> obs clamp  (tasks/base/vec_task.py:362-410,
 *                        tasks/ant.py:252-297) — no host synchronisation.
 *
 * Conventions
 *   - All tensors are device memory owned by the caller (PyTorch); pointers must
 *     stay valid for the call; layouts are the gym-visible ones:
 *       root_states (N*A, 13) f32 [px py pz qx qy qz qw vx vy vz wx wy wz]
 *       dof_state   (N*A*nD, 2) f32 [q, qdot];  sensors (N*A*S, 6) f32;
 *       dof_force   (N*A*nD) f32;  actions (N*A, nA) f32
 *       reset/progress/timeout buffers int64 (torch.long), as the reference.
 *   - Kernels are asynchronous on the caller's HIP stream (hipStream_t passed as
 *     void*; NULL = default stream).  No entry point synchronises the device.
 *   - Return 0 on success, a negative MG_E* code otherwise; mg_last_error()
 *     returns a thread-local message.  No C++ exception crosses the ABI.
 *   - One mg_sim per (process, device); calls on one handle are not thread-safe.
 */
#ifndef MIGYM_H
#define MIGYM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MG_VERSION 7

#define MG_MAX_NODES 40
#define MG_MAX_BODIES 40
#define MG_MAX_GEOMS 48
#define MG_MAX_PAIRS 192
#define MG_MAX_SENSORS 8
#define MG_MAX_TENDONS 8
#define MG_MAX_HAND_DOFS 32
#define MG_MAX_HULL_VERTS 160   /* the convex-mesh geom's hull (mg_model.hull_*) */
#define MG_MAX_HULL_PLANES 320

enum { MG_JT_FREE = 0, MG_JT_FIXED = 1, MG_JT_HINGE = 2, MG_JT_SLIDE = 3 };
enum { MG_GT_PLANE = 0, MG_GT_SPHERE = 1, MG_GT_CAPSULE = 2, MG_GT_BOX = 3, MG_GT_CYLINDER = 4, MG_GT_ELLIPSOID = 5,
       MG_GT_CONVEX = 6 /* convex mesh: the model's hull_* tables */ };
enum { MG_OK = 0, MG_EINVAL = -1, MG_EDEVICE = -2, MG_ENOMEM = -3, MG_ECAPACITY = -4 };
enum { MG_TASK_CARTPOLE = 0, MG_TASK_ANT = 1, MG_TASK_HUMANOID = 2, MG_TASK_SHADOW_HAND = 3 };
#define MG_MAX_AGENTS 8
enum { MG_SET_ROOT_STATE = 0, MG_SET_DOF_STATE = 1, MG_SET_DOF_TARGET = 2 };
/* coordinate space of applied rigid-body forces (gymapi.CoordinateSpace) */
enum { MG_ENV_SPACE = 0, MG_LOCAL_SPACE = 1, MG_GLOBAL_SPACE = 2 };
/* geom collision filter bits (mg_model.geom_filter) */
enum { MG_COLLIDE_GROUND = 1, MG_COLLIDE_OBJECT = 2 };

/* One articulation ("actor asset") as a dynamics tree of 1-DOF nodes.
 * Produced by migym/model.py (pack_model); field order == MODEL_DTYPE. */
typedef struct mg_model {
  int32_t num_nodes, num_dofs, fixed_base, num_bodies;
  int32_t num_geoms, num_pairs, num_sensors, nv;
  int32_t parent[MG_MAX_NODES];
  int32_t jtype[MG_MAX_NODES];
  int32_t limited[MG_MAX_NODES];
  int32_t node_body[MG_MAX_NODES];
  float t[MG_MAX_NODES][3];        /* joint anchor in parent node frame */
  float r0[MG_MAX_NODES][4];       /* rest rotation parent node -> node (xyzw) */
  float axis[MG_MAX_NODES][3];     /* joint axis, node frame (unit) */
  float mass[MG_MAX_NODES];
  float com[MG_MAX_NODES][3];      /* node frame */
  float inertia[MG_MAX_NODES][6];  /* about COM, node frame: xx yy zz xy xz yz */
  float armature[MG_MAX_NODES];
  float damping[MG_MAX_NODES];
  float stiffness[MG_MAX_NODES];
  float lower[MG_MAX_NODES];
  float upper[MG_MAX_NODES];
  int32_t body_node[MG_MAX_BODIES];
  int32_t body_parent[MG_MAX_BODIES];
  float body_pos[MG_MAX_BODIES][3];  /* body origin in its node frame */
  float body_quat[MG_MAX_BODIES][4];
  float body_com[MG_MAX_BODIES][3];  /* body COM in body frame */
  int32_t geom_type[MG_MAX_GEOMS];
  int32_t geom_node[MG_MAX_GEOMS];
  int32_t geom_body[MG_MAX_GEOMS];
  int32_t geom_filter[MG_MAX_GEOMS]; /* MG_COLLIDE_* bits */
  float geom_size[MG_MAX_GEOMS][3];
  float geom_pos[MG_MAX_GEOMS][3];   /* node frame */
  float geom_quat[MG_MAX_GEOMS][4];  /* node frame; capsule axis = local z */
  int32_t pair[MG_MAX_PAIRS][2];     /* self-collision geom pairs */
  int32_t sensor_body[MG_MAX_SENSORS];
  /* ---- position drives, fixed tendons and the free object of hand tasks
   * (shadow_hand.py:234-266, 684-698; shared.xml:55-72, 249-270) */
  float drive_kp[MG_MAX_NODES];      /* PD drive stiffness (MJCF <position kp>); > 0 = DOF_MODE_POS */
  float effort_limit[MG_MAX_NODES];  /* |drive force| limit (actuator forcerange) */
  int32_t num_tendons;
  int32_t gravity_off;               /* AssetOptions.disable_gravity of the articulation */
  int32_t tendon_dof[MG_MAX_TENDONS][2];
  float tendon_coef[MG_MAX_TENDONS][2];
  float tendon_range[MG_MAX_TENDONS][2];
  float tendon_limit_stiffness[MG_MAX_TENDONS];
  float tendon_damping[MG_MAX_TENDONS];
  /* One free rigid body per env next to the articulation (the manipulated object), plus a
   * kinematic goal actor.  Root-state rows per env are then [articulation, object, goal] and
   * rigid-body rows [articulation bodies..., object, goal]. */
  int32_t obj_type;                  /* 0 = none, MG_GT_BOX (block), MG_GT_ELLIPSOID (egg), MG_GT_CAPSULE (pen) */
  int32_t pair_mjcf;                 /* 1 = the pairs are explicit MJCF <pair>s (condim 1, margin 0): frictionless,
                                      * and in contact from zero distance (not the sim's contact offset) */
  float obj_mass;
  float obj_inertia[3];              /* principal moments, object frame (COM at the origin) */
  float obj_size[3];                 /* box half extents | ellipsoid semi-axes | capsule (radius, half length
                                      * along the object's z, 0) */
  float obj_lin_damping;
  float obj_ang_damping;
  float obj_gravity;                 /* 1 = the object falls under sim gravity */
  /* The convex-mesh collision geom (MG_GT_CONVEX; ShadowHand's robot0:C_forearm = mesh robot0:forearm_cvx,
   * robot.xml:8, shared_asset.xml:15), one per model: its hull in the geom frame (vertices, and outward
   * face planes n.x <= d inside).  geom_size of that geom = the hull's half extents about geom_pos. */
  int32_t hull_num_verts, hull_num_planes;
  float hull_vert[MG_MAX_HULL_VERTS][3];
  float hull_plane[MG_MAX_HULL_PLANES][4];
  /* Link velocity damping and cap of the articulation (gym AssetOptions.angular_damping /
   * max_angular_velocity; gym defaults 0.5 / 64: ant.py:152, humanoid.py:153-154, shadow_hand.py:240,
   * cartpole.py:86-87 keeps the defaults).  Damping acts on every link as the implicit couple
   * -c I_link w (a free link's w decays by 1/(1 + h c) per substep); the cap clamps every link's |w|
   * after the solve.  obj_max_ang_vel: the free object's cap (its damping is
   * obj_ang_damping).  A cap <= 0 disables it. */
  float link_ang_damping;
  float link_max_ang_vel;
  float obj_max_ang_vel;
  int32_t pad_model;
  /* Dry joint friction per DOF node: the MJCF joint `frictionloss` (the hand's default class, shared.xml:13:
   * 0.001), MuJoCo's constant friction torque bound, as the smooth law tau = -f tanh(qd / MG_FRICTIONLOSS_VS)
   * treated linearly implicitly like the damping (diagonal += h f / v_s sech^2); 0 = none */
  float frictionloss[MG_MAX_NODES];
} mg_model;
/* the regularization speed of the joint friction law (rad/s for hinges, m/s for slides) */
#define MG_FRICTIONLOSS_VS 0.01f

/* Simulation parameters (cfg['sim'] of the task YAML: Ant.yaml:42-61). */
typedef struct mg_sim_params {
  float dt;                 /* control dt (sim.dt) */
  int32_t substeps;         /* sim.substeps */
  float gravity[3];
  int32_t pos_iters;        /* physx.num_position_iterations: PGS sweeps per substep */
  float contact_offset;     /* physx.contact_offset: contacts generated below this gap */
  float rest_offset;        /* physx.rest_offset */
  float max_depen_vel;      /* physx.max_depenetration_velocity */
  float friction;           /* ground-plane friction coefficient */
  float baumgarte;          /* penetration recovery factor (build-defined) */
  float limit_margin;       /* joint-limit rows are built when within this distance */
  int32_t max_contacts;     /* per-actor contact capacity (<= MG_MAX_CONTACTS) */
  int32_t agents;           /* articulations per env (MA layouts; 1 otherwise) */
  int16_t solver_type;      /* MG_SOLVER_PGS (0, north_star) or MG_SOLVER_TGS (1, the reference's default,
                             * config.yaml:31): build-defined TGS, DESIGN.md §4 */
  int16_t vel_iters;        /* physx.num_velocity_iterations: TGS runs max(pos_iters, vel_iters) bias-free velocity
                             * sweeps after its sub-steps; unused by PGS.  (Two int16 keep the struct at 60 bytes:
                             * the kernels' argument layout, and so their code, stays as it was) */
} mg_sim_params;
#define MG_SOLVER_PGS 0
#define MG_SOLVER_TGS 1

/* Gym-visible state buffers the sim reads/writes (zero-copy, caller owned). */
typedef struct mg_state_views {
  float* root_states;       /* (N*A, 13) */
  float* dof_state;         /* (N*A*nD, 2) */
  const float* dof_actuation; /* (N*A*nD) effort, may be NULL (= zero) */
  float* sensors;           /* (N*A*S, 6), may be NULL */
  float* dof_force;         /* (N*A*nD), may be NULL */
  float* rigid_body_states; /* (N*A*nB, 13), may be NULL */
  const float* dof_targets; /* (N*A*nD) PD position targets (set_dof_position_target_tensor), may be NULL */
  /* gym.apply_rigid_body_force_tensors(sim, forces, None, space) (shadow_hand.py:700-708): forces
   * (N*A*nB, 3) in the rigid-body layout, applied at each body's centre of mass for every substep
   * of the next simulate.  Rows of the free object are applied; articulation rows must be zero.
   * NULL = no forces.  The fused hand step writes this tensor (it owns the random-force update). */
  float* rb_forces;
  int32_t rb_force_space;   /* MG_LOCAL_SPACE: body frame at the start of each substep; else world */
  int32_t env_props_stride; /* floats per row of env_props (mg_env_props_layout) */
  /* per-actor physical properties under domain randomization ((N*A, stride), see below); NULL = the
   * model's constants for every actor */
  const float* env_props;
  /* gym.acquire_net_contact_force_tensor / refresh_net_contact_force_tensor (franka_reach_MA.py:506, 563):
   * (N*A*nB, 3) in the rigid-body layout (hand tasks: the articulation's bodies, the object, the goal), the
   * world-frame net contact force on each body over the last substep (contact impulses / h; + on a contact's
   * side A, - on side B; the ground plane has no row).  Written by mg_sim_simulate and the fused step when bound;
   * NULL = not computed. */
  float* net_contact_forces;
} mg_state_views;

/* Task constants (cfg['env'] of the task YAML). */
typedef struct mg_task_params {
  int32_t task_id;          /* MG_TASK_* */
  int32_t num_obs;
  int32_t num_actions;
  int32_t max_episode_length;
  float dt;
  float clip_actions;       /* env.clipActions (inf if absent) */
  float clip_obs;           /* env.clipObservations (inf if absent) */
  float power_scale;        /* env.powerScale; Cartpole: maxEffort */
  float dof_vel_scale;
  float angular_velocity_scale;
  float contact_force_scale;
  float heading_weight;
  float up_weight;
  float actions_cost_scale;
  float energy_cost_scale;
  float joints_at_limit_cost_scale;
  float death_cost;
  float termination_height;
  float max_motor_effort;
  float reset_dist;         /* Cartpole resetDist */
  float target[3];          /* walk target (ant.py:105) */
  float start_pos[3];       /* actor start pose (ant.py:163-166) */
  float start_rot[4];
  float motor_effort[64];   /* per-DOF gear (actuator order, applied by DOF position) */
  float dof_lower[64];      /* task-side dof limits (swapped if lower>upper, ant.py:199-206) */
  float dof_upper[64];
  float initial_dof_pos[64];
  /* multi-agent layout (SURVEY.md §8(a) A-MA; franka_reach_MA.py:22-38, 598-612, 875-889):
   * actors are env-major (actor = env * num_agents + agent); an env resets only when all
   * of its agents are done (AND filter); obs rows append the other agents' torso positions
   * relative to self in cyclic-shift order.  num_agents = 1 for single-agent tasks. */
  int32_t num_agents;
  /* env.controlFrequencyInv: gym.simulate runs this many times per VecTask.step (vec_task.py:381-384)
   * while pre_physics_step / post_physics_step run once; 0 is taken as 1 */
  int32_t control_freq_inv;
  float agent_offset[8][3]; /* start-pose / target offset of each agent within its env */
  /* in-hand manipulation (MG_TASK_SHADOW_HAND; tasks/shadow_hand.py:40-118, ShadowHand.yaml) */
  int32_t num_fingertips;
  int32_t fingertip_body[8];          /* gym rigid-body index of each fingertip */
  int32_t actuated_dof[MG_MAX_HAND_DOFS]; /* action column -> DOF (actuator order) */
  int32_t max_consecutive_successes;
  int32_t use_relative_control;
  int32_t ignore_z_rot;               /* pen */
  int32_t obs_type;                   /* 0 full_state (211), 1 full (157), 2 full_no_vel (77), 3 openai (42) */
  int32_t rb_per_env;                 /* rigid-body rows per env (articulation bodies + object + goal) */
  int32_t num_dofs;                   /* hand DOFs (dof_state rows per env) */
  float dof_speed_scale;
  float act_moving_average;
  float dist_reward_scale;
  float rot_reward_scale;
  float rot_eps;
  float action_penalty_scale;
  float success_tolerance;
  float reach_goal_bonus;
  float fall_dist;
  float fall_penalty;
  float av_factor;
  float vel_obs_scale;
  float force_torque_obs_scale;
  float reset_position_noise;
  float reset_dof_pos_noise;
  float reset_dof_vel_noise;
  float object_start[3];             /* object_init_state position */
  float goal_displacement[3];        /* goal actor = goal_states + displacement */
  float goal_dz;                     /* goal_init = object_init + (0, 0, goal_dz) */
  /* asymmetric actor-critic (shadow_hand.py:125-131, 470-471): states_buf = the full_state layout */
  int32_t num_states;                /* 0 = no states buffer, else 211 */
  /* random object forces (shadow_hand.py:69-72, 196-199, 641-643, 700-708); force_scale 0 = off */
  int32_t object_rb;                 /* rigid-body row of the object within an env (object_rb_handles) */
  float force_scale;
  float force_decay_step;            /* forceDecay ** (dt / forceDecayInterval), fp32 (torch.pow) */
  float force_prob_lo;               /* forceProbRange */
  float force_prob_hi;
  float object_rb_mass;              /* object_rb_masses */
  /* observation column -> (segment << 8 | index) of the observationType layout (obs_map) and of the
   * full_state layout (state_map).  Filled by the library before a hand-task launch; callers need
   * not set them. */
  uint16_t obs_map[256];
  uint16_t state_map[256];
} mg_task_params;

/* Task-layer buffers (VecTask.allocate_buffers, vec_task.py:302-325). */
typedef struct mg_task_buffers {
  const float* actions;     /* (N*A, nA) raw policy actions (clamped inside) */
  float* actions_out;       /* (N*A, nA) clamped actions kept for obs (self.actions), may == NULL */
  float* obs;               /* (N*A, nO) obs_buf (unclamped, like the reference) */
  float* obs_clamped;       /* (N*A, nO) obs_dict['obs'] = clamp(obs_buf), may be NULL */
  float* rew;               /* (N*A) */
  int64_t* reset;           /* (N*A) */
  int64_t* progress;        /* (N*A) */
  uint8_t* timeout;         /* (N*A) torch.bool, like VecTask.timeout_buf after step */
  float* potentials;        /* (N*A) */
  float* prev_potentials;   /* (N*A) */
  float* up_vec;            /* (N*A, 3) */
  float* heading_vec;       /* (N*A, 3) */
  const float* noise;       /* (N*A, 2*nD) injected U(0,1) reset noise, or NULL = device RNG;
                             * ShadowHand: (N, 66) = [goal-only draw 4 | reset_idx draw 53 |
                             * reset_target_pose draw 4 | force-probability redraw 1 (U(0,1)) |
                             * force selection 1 (U(0,1)) | force direction 3 (N(0,1))]
                             * (shadow_hand.py:587, 610, 642-643, 704-706) */
  uint64_t seed;            /* device RNG seed (counter-based, keyed by global env id) */
  uint64_t step_counter;    /* VecTask.control_steps: RNG counter */
  int64_t env_offset;       /* global id of this shard's first env (multi-GPU); the RNG key of local actor a
                             * is the global actor id env_offset * num_agents + a, so a rollout does not
                             * depend on how the envs are sharded */
  /* in-hand manipulation (tasks/shadow_hand.py:186-219); unused by the other tasks */
  float* prev_targets;      /* (N, nD) */
  float* goal_states;       /* (N, 13) */
  int64_t* reset_goal;      /* (N) reset_goal_buf */
  float* successes;         /* (N) */
  float* consecutive_successes; /* (1) running mean (shadow_hand.py:795-798) */
  uint64_t* reduce_scratch; /* (2) device scratch: sum(resets), sum(successes * resets) */
  float* states;            /* (N, num_states) states_buf, may be NULL */
  float* random_force_prob; /* (N) per-env force probability, redrawn on reset; may be NULL */
  /* multi-GPU output path: when set, the step also writes each actor's row
   * [clamped obs (nO) | rew | reset] into this (N*A, nO + 2) f32 buffer, the message the obs gather
   * sends (migym/dist.py); the caller double-buffers it so the gather of step k overlaps step k+1 */
  float* out_pack;
  /* ShadowHand: 1 = leave this step's running-mean partial sums in reduce_scratch (the caller
   * all-reduces them over the ranks, then calls mg_hand_finalize); 0 = apply them in the step */
  int32_t defer_finalize;
  int32_t pad_tb;
} mg_task_buffers;

typedef struct mg_sim mg_sim;

/* ---- domain randomization (tasks/base/vec_task.py:612-842, utils/dr_utils.py) ----
 * The reference re-sets actor properties through the gym property setters in a per-env Python loop.
 * Here the per-actor physical properties live in one device table, env_props (N*A rows of `stride`
 * floats, bound through mg_state_views.env_props), which mg_dr_apply rewrites for the actors being
 * randomized and the physics kernels read instead of the model's constants.  Row layout (offsets
 * from mg_env_props_layout):
 *   MG_EP_NODE    num_nodes x MG_EP_NODE_WIDTH (9): [mass, armature, damping, stiffness, lower, upper, drive kp,
 *                 effort, frictionloss]
 *                 (mass of the node's body; its inertia scales with mass / model mass:
 *                 set_actor_rigid_body_properties(..., recomputeInertia=True))
 *   MG_EP_GEOM    num_geoms: friction of each collision shape (a contact's friction is the mean of
 *                 its two shapes'; the ground plane's is mg_sim_params.friction)
 *   MG_EP_TENDON  num_tendons x 2: [limit stiffness, damping]
 *   MG_EP_OBJECT  4: [mass, friction, scale, 0] of the free object (scale: half extents x s,
 *                 mass x s^3, inertia x s^5) */
enum { MG_EP_NODE = 0, MG_EP_GEOM = 1, MG_EP_TENDON = 2, MG_EP_OBJECT = 3 };
#define MG_EP_NODE_WIDTH 9
enum { MG_DR_UNIFORM = 0, MG_DR_GAUSSIAN = 1, MG_DR_LOGUNIFORM = 2 };
enum { MG_DR_ADDITIVE = 0, MG_DR_SCALING = 1 };
enum { MG_DR_SCHED_NONE = 0, MG_DR_SCHED_LINEAR = 1, MG_DR_SCHED_CONSTANT = 2 };

/* one randomized attribute (dr_utils.generate_random_samples / apply_random_samples) */
typedef struct mg_dr_desc {
  int32_t distribution;     /* MG_DR_UNIFORM / GAUSSIAN (range = [mu, std]) / LOGUNIFORM */
  int32_t operation;        /* MG_DR_ADDITIVE / MG_DR_SCALING */
  int32_t schedule;         /* MG_DR_SCHED_* */
  int32_t schedule_steps;
  int32_t num_buckets;      /* > 0: get_bucketed_val over the unscheduled range */
  int32_t after_setup;      /* 0: its property holds a setup_only attribute (randomized on the first call only) */
  float range[2];
} mg_dr_desc;
/* one element of an attribute: env_props column, descriptor, original value (og_prop) */
typedef struct mg_dr_attr {
  int32_t slot;
  int32_t desc;
  float og;
  int32_t pad;
} mg_dr_attr;

typedef struct mg_dr_apply_args {
  const mg_dr_desc* descs;  /* device */
  const mg_dr_attr* attrs;  /* device, nattr */
  int32_t nattr;
  int32_t stride;           /* env_props row length */
  int32_t n;                /* actors */
  int32_t frequency;        /* randomization_params.frequency */
  int32_t first;            /* first_randomization: every actor, setup_only attributes included */
  int32_t increment;        /* randomize_buf += 1 before the test (post_physics_step's increment) */
  int64_t last_step;        /* gym.get_frame_count (schedules) */
  float* env_props;         /* (n, stride) */
  const int64_t* reset_mask;/* (n) reset_buf of the resetting step (ignored with first) */
  int64_t* randomize_buf;   /* (n) */
  const float* samples;     /* (n, nattr) injected samples (generate_random_samples output), or NULL */
  uint64_t seed;            /* device RNG: counter-based, keyed by (global actor id, counter, attr) */
  uint64_t counter;
  int64_t env_offset;
} mg_dr_apply_args;

/* noise_lambda of randomization_params.observations / .actions (vec_task.py:684-720), in the
 * reference's fp32 operation order:
 *   x = op(x, ((corr * c_scale + c_shift) + z * scale) + shift)
 * gaussian: z ~ N(0,1), scale = var, shift = mu, c_scale = var_corr, c_shift = mu_corr;
 * uniform:  z ~ U(0,1), scale = hi - lo, shift = lo, c_scale = hi_corr - lo_corr, c_shift = lo_corr
 * (corr is N(0,1) in both, as the reference draws it with randn_like).  Optional clamp into x_clamped. */
typedef struct mg_dr_noise_args {
  float* x;                 /* (n) in/out */
  float* x_clamped;         /* (n) clamp(x, +-clip) or NULL */
  float clip;
  int32_t distribution;     /* MG_DR_GAUSSIAN or MG_DR_UNIFORM */
  int32_t operation;        /* MG_DR_ADDITIVE / MG_DR_SCALING */
  int32_t refresh_corr;     /* draw a new corr tensor first ("corr" absent from dr_randomizations) */
  float* corr;              /* (n) persistent correlated noise */
  int64_t n;
  float scale, shift;       /* schedule applied by the caller */
  float c_scale, c_shift;
  const float* injected;    /* (n) per-call draws (randn_like / rand_like), or NULL = device RNG */
  const float* injected_corr; /* (n) corr draws when refreshing, or NULL */
  uint64_t seed;
  uint64_t counter;
  int64_t elem_offset;      /* global index of element 0 (multi-GPU shards) */
  uint32_t key;             /* RNG stream of this tensor */
  int32_t pad;
} mg_dr_noise_args;

int mg_env_props_layout(const mg_model* m, int32_t offsets[4]);   /* returns the row stride (floats) */
int mg_env_props_defaults(const mg_model* m, float* row);           /* host: one row of model values */
int mg_dr_apply(const mg_dr_apply_args* a, void* stream);
int mg_dr_noise(const mg_dr_noise_args* a, void* stream);
/* replace the simulation parameters (gym.set_sim_params; DR of sim_params.gravity) */
int mg_sim_set_params(mg_sim* sim, const mg_sim_params* params);

const char* mg_last_error(void);
int mg_version(void);
size_t mg_model_sizeof(void);
size_t mg_task_params_sizeof(void);
size_t mg_task_buffers_sizeof(void);
size_t mg_sim_params_sizeof(void);
size_t mg_state_views_sizeof(void);
size_t mg_dr_desc_sizeof(void);
size_t mg_dr_apply_args_sizeof(void);
size_t mg_dr_noise_args_sizeof(void);
/* profiling aid (phase-timing build only, see isaacgymenvs-ma_amd/build.py --timing): MG_NUM_PHASES counters */
#define MG_NUM_PHASES 32
int mg_debug_phase_cycles(uint64_t* out, int32_t reset);
/* ... and the per-item rows behind it (an item = one wave's teams; cap items of MG_NUM_PHASES counts each) */
int mg_debug_phase_waves(uint64_t* out, int32_t cap);

int mg_sim_create(const mg_model* model, const mg_sim_params* params, int32_t num_envs, int32_t device,
                  mg_sim** out);
int mg_sim_bind(mg_sim* sim, const mg_state_views* views);
int mg_sim_simulate(mg_sim* sim, void* stream);
int mg_sim_destroy(mg_sim* sim);

/* Scatter rows of `src` (same layout as the bound buffer) into the bound
 * buffer for the actor indices idx[0..n) (int32, global actor ids). */
int mg_set_indexed(mg_sim* sim, int32_t which, const float* src, const int32_t* idx, int32_t n, void* stream);

/* Reference jit functions, one thread per env. Inputs/outputs as in the
 * reference signatures; `root_states` etc. may alias the sim buffers. */
int mg_compute_observations(const mg_task_params* tp, int32_t n, const float* root_states, const float* dof_state,
                            const float* dof_force, const float* sensors, const float* actions,
                            float* potentials, float* prev_potentials, float* up_vec, float* heading_vec,
                            float* obs, void* stream);
int mg_compute_reward(const mg_task_params* tp, int32_t n, const float* obs, const float* actions,
                      const float* potentials, const float* prev_potentials, const int64_t* progress,
                      int64_t* reset, float* rew, void* stream);

/* Task-layer half of VecTask.step before the physics (pre_physics_step after the action
 * clamp): locomotion -> dof_actuation = clamp(a) * gear * power_scale (ant.py:281-285);
 * ShadowHand -> masked goal/env resets + PD targets into views->dof_targets
 * (shadow_hand.py:670-698).  sim == NULL: `views` are used. */
int mg_pre_physics(mg_sim* sim, const mg_task_params* tp, const mg_state_views* views,
                   const mg_task_buffers* tb, int32_t n, void* stream);

/* Task-layer half of VecTask.step after the physics (post_physics_step +
 * timeout + obs clamp).  With `sim`==NULL the state views in `views` are used
 * as the post-physics state (physics-free replay, parity tests). */
int mg_post_physics(mg_sim* sim, const mg_task_params* tp, const mg_state_views* views,
                    const mg_task_buffers* tb, int32_t n, void* stream);

/* ShadowHand: apply the consecutive_successes running mean (shadow_hand.py:795-798) from the partial
 * sums in tb->reduce_scratch and clear them.  Only needed with tb->defer_finalize (multi-GPU: the caller
 * all-reduces reduce_scratch over the ranks first, so every rank holds the whole-node mean). */
int mg_hand_finalize(const mg_task_params* tp, const mg_task_buffers* tb, void* stream);

/* reset_idx(env_ids) applied immediately (ant.py:252-279, humanoid.py:251-278, cartpole.py:122-136,
 * shadow_hand.py:586-668): for the n ids in `ids` (int32 device array; locomotion / MA: actor rows of
 * reset_buf, ShadowHand: envs), write the reset DOF state (noise), root row, potentials (locomotion) or
 * goal, object pose, hand DOFs and PD targets (ShadowHand), and clear progress / reset / successes --
 * the state a caller reads right after the reference's reset_idx.  Noise: the counter RNG on its own
 * stream (seed, global env id, tb->step_counter | 2^62), or tb->noise rows indexed like the step's.
 * The fused step keeps applying reset_buf's masked resets itself; this entry serves callers that reset
 * outside the step (evaluation, curricula). */
int mg_reset_idx(mg_sim* sim, const mg_task_params* tp, const mg_task_buffers* tb, const int32_t* ids, int32_t n,
                 void* stream);

/* Whole VecTask.step: actions -> actuation -> simulate -> post_physics.  Launches of one sim must be
 * stream-ordered: the multi-wave kernel instances dequeue work items from the sim's device counters,
 * which the last wave of each launch zeroes for the next. */
int mg_env_step(mg_sim* sim, const mg_task_params* tp, const mg_task_buffers* tb, void* stream);

/* Physics-bypass replay of mg_env_step (test infrastructure: pins the fused kernels' own task layer
 * to the reference's fake-gym traces).  The kernel instance mg_env_step launches is
 * run with its whole task layer (action clamp, actuation / PD targets, masked resets, observations,
 * reward, running mean, write-back), but gym.simulate is replaced by the state given here, exactly
 * as the traces' fake gym.simulate overwrites the sim state (tests/golden/make_traces.py). */
typedef struct mg_replay {
  const float* root_states;       /* (N*A*R, 13) post-simulate root rows; hand tasks (R = 3): the object
                                   * row is taken (hand and goal actors are not simulated) */
  const float* dof_state;         /* (N*A*nD, 2) */
  const float* sensors;           /* (N*A*S, 6) or NULL (zeros) */
  const float* dof_force;         /* (N*A*nD) or NULL (zeros) */
  const float* rigid_body_states; /* hand tasks: (N, nB + 2, 13); the articulation rows are taken */
  float* pre_root_states;         /* out or NULL: root rows after pre_physics_step (what simulate starts from) */
  float* pre_dof_state;           /* out or NULL: DOF state after pre_physics_step */
} mg_replay;
int mg_env_step_replay(mg_sim* sim, const mg_task_params* tp, const mg_task_buffers* tb, const mg_replay* rp,
                       void* stream);

/* Measurement aid (no reference counterpart; bench.py's roofline.kernel_ms): the device-side duration of the
 * fused step kernel, from the first wave's start to the last wave's end on the GPU's constant wall clock
 * (wall_clock64, hipDeviceAttributeWallClockRate), so that no launch, queue or event-packet overhead is in it.
 * mg_kernel_span_begin(sim, cap): the next `cap` mg_env_step launches of `sim` record their span (one slot each;
 * 0 turns recording off; the kernels run unchanged otherwise).  mg_kernel_span_read(sim, ms, cap, &n):
 * synchronises the device and returns the recorded spans in milliseconds, in launch order. */
int mg_kernel_span_begin(mg_sim* sim, int32_t cap);
int mg_kernel_span_read(mg_sim* sim, double* ms, int32_t cap, int32_t* n_out);
/* mg_kernel_span_waves(sim, launch, out, cap, &n): the raw per-wave (start, end) GPU wall-clock ticks of recorded
 * launch `launch` (out: 2 * cap uint64; n = the launch's waves, at most cap; ticks at hipDeviceAttributeWallClockRate
 * kHz) -- the launch's tail and dispatch ramp for tools/span_diag.py --waves */
int mg_kernel_span_waves(mg_sim* sim, int32_t launch, uint64_t* out, int32_t cap, int32_t* n_out);

/* Test aid (no reference counterpart): the work ordering's state.  mg_work_order(sim, order, cost,
 * cap, &mode, &n): synchronises the device; mode = 0 off, 1 lists, 2 sort; under the sort n = the env units (envs,
 * an MA env's agents counted once), `order` (n int32, or NULL) = the permutation the last mg_env_step ran in (slot ->
 * unit; the identity before the first sort) and `cost` (n uint8, or NULL) = the row counts that launch wrote (the
 * next sort's keys); at most cap entries are copied.  Off and lists report n = 0. */
int mg_work_order(mg_sim* sim, int32_t* order, uint8_t* cost, int32_t cap, int32_t* mode, int32_t* n_out);
/* Diagnostic (no reference counterpart): the step-kernel instance the dispatcher picked for `sim`:
 * team_lanes = lanes per actor (T), compact = 1 for the 12-waves-per-CU compact team layout, 0 for the classic one
 * (MIGYM_LAYOUT = auto | compact | classic, read at mg_sim_create). */
int mg_sim_kernel_layout(mg_sim* sim, int32_t* team_lanes, int32_t* compact);

#ifdef __cplusplus
}
#endif
#endif /* MIGYM_H */
