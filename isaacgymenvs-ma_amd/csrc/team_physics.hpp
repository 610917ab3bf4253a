// team_physics.hpp — gym.simulate on gfx950 with one *team* of T lanes per actor
// (SURVEY.md §8(a) rows A3-A9).  Same algorithm as physics.hpp/the oracle
// (ABA + speculative contacts + PGS + semi-implicit Euler),
// mapped onto a 64-wide wave so that nothing spills to scratch:
//
//   lane roles inside a team (tl = lane % T):
//     * generalized-velocity column j = tl  (nu_j lives in lane j's registers;
//       free base: j < 6 are the root twist [w; v_o], j >= 6 the joints)
//     * tree node: node i >= 1 lives on lane col(i) = (free ? 5 : -1) + i, the
//       root node on lane 0.  A node's kinematics (R, x, S, V), articulated
//       inertia (21 floats) and ABA factors (U, 1/D) stay in its lane.
//   tree recursions (FK, ABA backward/forward) are level-synchronous: nodes
//   of one depth compute together and publish what children/parents need in
//   the team's LDS tile; the per-child articulated-inertia contributions are
//   summed by the parent lane from LDS (deterministic order, no atomics).
//   contact generation: lane per geom / per self-pair, compaction by a team
//   prefix scan (shuffles), preserving the oracle's contact order.
//   constraint rows: the response column Y_r = M~^-1 J_r^T is produced by a
//   test-force ABA solve whose output lands distributed — lane j keeps
//   Y_r[j] in a register (Ycol[r]); PGS row updates are then a team dot
//   product (butterfly shuffles) plus one FMA per lane.
// All lanes of a wave run every phase (teams never diverge on barriers); a team's
// phases synchronise its wave (wsync), never the block: a block is W waves sharing one model tile.
//
// Hand tasks (OBJ = true, SURVEY.md §8(a) A4-A8 for ShadowHand): PD position drives
// (implicit toward the target, +-effort when saturated), fixed tendons (explicit soft
// limits), and a free rigid box whose 6 velocity columns [w; v_com] live on the lanes
// right after the articulation's; contacts between articulation geoms and the box
// couple the two blocks only through the PGS rows (response = ABA test solve on the
// articulation lanes + the box's closed-form inverse inertia on the object lanes).
#pragma once
#include "../../include/migym.h"
#include "convex.hpp"
#include "device_math.hpp"
#include "hull.hpp"
#include "common.hpp"

#include <type_traits>

namespace mg {

// The physics may contract a * b + c into FMAs (the oracle it is checked against is fp64; the task layer's
// reference arithmetic in task.hpp / hand_task.hpp keeps contraction off).  The caller's FP state is
// restored at the end of this header.
#pragma float_control(push)
#ifndef MG_PHYS_CONTRACT
#define MG_PHYS_CONTRACT 1  // 0: no FMA contraction in the physics (a parity A/B only)
#endif
#if MG_PHYS_CONTRACT
#pragma clang fp contract(fast)
#else
#pragma clang fp contract(off)
#endif
// per-phase contraction switches (parity A/B: which phase's FMA contraction moves the results off the fp64 oracle;
// MG_NOCONTRACT_MASK bits: 1 PGS visit, 2 ABA, 4 test solves, 8 FK, 16 integrate + velocity cap, 32 row Jacobians)
#ifndef MG_NOCONTRACT_MASK
#define MG_NOCONTRACT_MASK 0
#endif
#define MG_NC_OFF _Pragma("clang fp contract(off)")
// PGS visit products kept out of FMAs: 1 the velocity update nu += Y dl (the default, round 6), 2 the impulse update.
// Fusing the velocity update moved the DOF velocities off the fp64 oracle: the fraction of them within north_star's
// 1e-4 relative fell 0.8 % below the oracle's own fp32 build (Ant 16,384 / 65,536, MA-Ant), against 0.25 % unfused
// (the per-phase A/B: only this product matters; profiles/r06/ab_pgs_fusion.txt); it costs Ant 65,536 1.3 %
#ifndef MG_PGS_UNFUSE
#define MG_PGS_UNFUSE 1
#endif
#if MG_NOCONTRACT_MASK & 1
#define MG_NC_PGS MG_NC_OFF
#else
#define MG_NC_PGS
#endif
#if MG_NOCONTRACT_MASK & 2
#define MG_NC_ABA MG_NC_OFF
#else
#define MG_NC_ABA
#endif
#if MG_NOCONTRACT_MASK & 4
#define MG_NC_TS MG_NC_OFF
#else
#define MG_NC_TS
#endif
#if MG_NOCONTRACT_MASK & 8
#define MG_NC_FK MG_NC_OFF
#else
#define MG_NC_FK
#endif
#if MG_NOCONTRACT_MASK & 16
#define MG_NC_INT MG_NC_OFF
#else
#define MG_NC_INT
#endif
#if MG_NOCONTRACT_MASK & 32
#define MG_NC_JAC MG_NC_OFF
#else
#define MG_NC_JAC
#endif

// Block-shared LDS copy of the model tables the hot loops read ("model tile"):
// every per-node / per-geom constant is an LDS read (~64 cycles) instead of a dependent global load.
// Rows padded to odd strides.  The image is built once on the host (build_tile, at mg_sim_create) and
// each block copies it with 16-byte loads; the W waves of a block share one copy.
// vertices of the convex hull the LDS model tile holds: the block / pen instances, whose exact hull candidates
// (hull.hpp) read them in every GJK support; the egg tests the hull's planes only (global memory)
constexpr int tile_hull_verts(int obj) { return (obj == MG_GT_BOX || obj == MG_GT_CAPSULE) ? MG_MAX_HULL_VERTS : 1; }

template <int MN, int MG, int MP, int HV = 1>  // HV: hull vertex capacity of the tile (tile_hull_verts)
struct alignas(16) ModelTile {
  int parent[MN], jtype[MN], limited[MN];
  unsigned long long children[MN];
  unsigned long long anc[MN];   // ancestor mask of each node (itself and the root included)
  int lvs[MN];                  // the node's index among the nodes of its depth (compact layout's ABA slot)
  float nf[MN][33];   // 0-8 Rr0, 9-11 t, 12-14 axis, 15-17 com, 18-23 inertia, 24 mass, 25 arm, 26 damp,
                      // 27 stiff, 28 lower, 29 upper, 30 drive kp, 31 effort limit, 32 frictionloss
  int gtype[MG], gnode[MG], gbody[MG], gfil[MG];
  int tdof[MG_MAX_TENDONS][2];
  float tf[MG_MAX_TENDONS][6];   // coef0, coef1, lo, hi, limit stiffness, damping
  int nten;
  float gf[MG][17];   // 0-2 pos, 3-11 R, 12-14 size, 15 bounding radius
  int pairs[MP > 0 ? MP : 1][2];
  int nn, ng, np;
  int hnv;            // vertices of the convex-mesh geom's hull (mg_model.hull_*), 0 if none
  int hullg;          // the convex-mesh geom (-1 if none)
  int ground_round;   // every ground-colliding geom is a sphere or a capsule (one-pass ground contacts)
  // block / pen instances: the hull's vertices and their centroid for the exact hull candidates (hull.hpp), read
  // by every GJK support; its planes stay in global memory (one pass per call)
  float hv[HV][3];
  float hctr[4];
};

// host: the finished tile image of model m (child masks, rest rotations as matrices, geom frames)
template <int MN, int MG, int MP, int HV>
__host__ __device__ void build_tile(ModelTile<MN, MG, MP, HV>* t, const mg_model* m, int tid = 0, int nt = 1) {
  const int nn = m->num_nodes < MN ? m->num_nodes : MN, ng = m->num_geoms < MG ? m->num_geoms : MG;
  const int np = m->num_pairs < MP ? m->num_pairs : MP;
  for (int i = tid; i < nn; i += nt) {
    t->parent[i] = m->parent[i];
    t->jtype[i] = m->jtype[i];
    t->limited[i] = m->limited[i];
    unsigned long long ch = 0ull;
    for (int k = 1; k < nn; k++)
      if (m->parent[k] == i) ch |= 1ull << k;
    t->children[i] = ch;
    unsigned long long an = 1ull;
    int di = 0;
    for (int k = i; k > 0; k = m->parent[k]) {
      an |= 1ull << k;
      di++;
    }
    t->anc[i] = an;
    int lv = 0;  // nodes of the same depth before this one
    for (int k = 1; k < i; k++) {
      int dk = 0;
      for (int j = k; j > 0; j = m->parent[j]) dk++;
      lv += dk == di ? 1 : 0;
    }
    t->lvs[i] = i > 0 ? lv : 0;
    float* f = t->nf[i];
    const M3 R0 = quat_to_mat(m->r0[i][0], m->r0[i][1], m->r0[i][2], m->r0[i][3]);
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) f[3 * a + b] = R0.m[a][b];
    for (int k = 0; k < 3; k++) { f[9 + k] = m->t[i][k]; f[12 + k] = m->axis[i][k]; f[15 + k] = m->com[i][k]; }
    for (int k = 0; k < 6; k++) f[18 + k] = m->inertia[i][k];
    f[24] = m->mass[i]; f[25] = m->armature[i]; f[26] = m->damping[i]; f[27] = m->stiffness[i];
    f[28] = m->lower[i]; f[29] = m->upper[i];
    f[30] = m->drive_kp[i]; f[31] = m->effort_limit[i];
    f[32] = m->frictionloss[i];
  }
  const int nten = m->num_tendons < MG_MAX_TENDONS ? m->num_tendons : MG_MAX_TENDONS;
  for (int q = tid; q < nten; q += nt) {
    t->tdof[q][0] = m->tendon_dof[q][0];
    t->tdof[q][1] = m->tendon_dof[q][1];
    t->tf[q][0] = m->tendon_coef[q][0]; t->tf[q][1] = m->tendon_coef[q][1];
    t->tf[q][2] = m->tendon_range[q][0]; t->tf[q][3] = m->tendon_range[q][1];
    t->tf[q][4] = m->tendon_limit_stiffness[q]; t->tf[q][5] = m->tendon_damping[q];
  }
  for (int g = tid; g < ng; g += nt) {
    t->gtype[g] = m->geom_type[g];
    t->gnode[g] = m->geom_node[g];
    t->gbody[g] = m->geom_body[g];
    t->gfil[g] = m->geom_filter[g];
    float* f = t->gf[g];
    const M3 Rg = quat_to_mat(m->geom_quat[g][0], m->geom_quat[g][1], m->geom_quat[g][2], m->geom_quat[g][3]);
    for (int k = 0; k < 3; k++) { f[k] = m->geom_pos[g][k]; f[12 + k] = m->geom_size[g][k]; }
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) f[3 + 3 * a + b] = Rg.m[a][b];
    const float* sz = m->geom_size[g];
    const int ty = m->geom_type[g];
    f[15] = (ty == MG_GT_BOX || ty == MG_GT_CONVEX) ? sqrtf(sz[0] * sz[0] + sz[1] * sz[1] + sz[2] * sz[2])
                            : (ty == MG_GT_CAPSULE ? sz[0] + sz[1] : sz[0]);
  }
  for (int q = tid; q < np; q += nt) {
    t->pairs[q][0] = m->pair[q][0];
    t->pairs[q][1] = m->pair[q][1];
  }
  if (tid == 0) {
    t->nn = nn; t->ng = ng; t->np = np; t->nten = nten; t->hnv = m->hull_num_verts;
    t->ground_round = 1;
    for (int g = 0; g < ng; g++)
      if ((m->geom_filter[g] & MG_COLLIDE_GROUND) && m->geom_type[g] != MG_GT_SPHERE && m->geom_type[g] != MG_GT_CAPSULE)
        t->ground_round = 0;
    // the convex-mesh geom that collides with the object (mg_sim_create allows one), else the lowest one
    t->hullg = -1;
    for (int g = ng - 1; g >= 0; g--)
      if (m->geom_type[g] == MG_GT_CONVEX) t->hullg = g;
    for (int g = ng - 1; g >= 0; g--)
      if (m->geom_type[g] == MG_GT_CONVEX && (m->geom_filter[g] & MG_COLLIDE_OBJECT)) t->hullg = g;
    t->hctr[0] = t->hctr[1] = t->hctr[2] = t->hctr[3] = 0.0f;
    if (HV > 1 && m->hull_num_verts > 0 && m->hull_num_verts <= HV) {
      float cx = 0.0f, cy = 0.0f, cz = 0.0f;
      for (int v = 0; v < m->hull_num_verts; v++) {
        for (int k = 0; k < 3; k++) t->hv[v][k] = m->hull_vert[v][k];
        cx += m->hull_vert[v][0];
        cy += m->hull_vert[v][1];
        cz += m->hull_vert[v][2];
      }
      t->hctr[0] = cx / (float)m->hull_num_verts;
      t->hctr[1] = cy / (float)m->hull_num_verts;
      t->hctr[2] = cz / (float)m->hull_num_verts;
    }
  }
}

// device: the block copies the prebuilt image (global) into its LDS tile, 16 bytes per lane and load
template <class MT>
__device__ __forceinline__ void copy_tile(MT* t, const MT* img) {
  static_assert(sizeof(MT) % 16 == 0, "the tile is copied in 16-byte pieces");
  const uint4* src = reinterpret_cast<const uint4*>(img);
  uint4* dst = reinterpret_cast<uint4*>(t);
  for (int i = threadIdx.x; i < (int)(sizeof(MT) / 16); i += blockDim.x) dst[i] = src[i];
}

// Teams never span a wave, so the team phases synchronise their own wave only (rocPRIM's wave_barrier:
// a wave's LDS operations complete in order; the wavefront-scope fences keep the compiler from moving
// LDS accesses across the point).  No s_barrier: the other waves of the block run on independently.
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

static_assert(MG_MAX_GEOMS < 128 && MG_MAX_NODES < 128, "contact sides are packed as int8");
constexpr float kBoxBlend = 1e-3f;  // point_box: the band (m) over which an interior point's normal blends faces

// PGS visits per block of the sweep (their data are loaded one block ahead; 2 and 8 measured slower)
constexpr int kPgsPrefetch = 4;
// rows whose (J, Y) columns stay in registers; the rest live in private (scratch) arrays (same-box A/B vs 16:
// Ant +0.8 %, Humanoid +0.8 %, ShadowHand +0.6 %; 8 and 20 slower).  The egg keeps every row in scratch.
#ifndef MG_KJY
#define MG_KJY 12
#endif
#ifndef MG_KJY_LOCO32
#define MG_KJY_LOCO32 16
#endif
#ifndef MG_KJY_EGG
#define MG_KJY_EGG 0
#endif
#ifndef MG_KJY_HAND
#define MG_KJY_HAND 12  // block / pen
#endif
constexpr int kJYRegs = MG_KJY;
// test-solve columns per batch (a multiple of 3).  16-lane teams: 6 (round 6, with the compact layout at three waves
// per SIMD and 168 VGPRs: the per-batch arrays of 12 columns spilled; same box, two passes, Ant 65,536 177.0 ->
// 201.1 M env-steps/s, 32,768 161.0 -> 180.2 M, 16,384 124.8 -> 137.9 M, MA-Ant 8,192 39.5 -> 43.4 M; 3 columns 186.4 /
// 167.1 / 125.4 / 39.7 M, 9 columns 195.0 M at 65,536; profiles/r06/ab_rb.txt.  At two waves per SIMD 12 had
// beaten 6: +0.7 % Ant).  32-lane locomotion teams: 12 (9 or 18: -5 % / -34 %); Cartpole 6
#ifndef MG_RB_LOCO16
#define MG_RB_LOCO16 6
#endif
constexpr int kRBLoco = MG_RB_LOCO16;
#ifndef MG_RB_LOCO32
#define MG_RB_LOCO32 12  // the 32- and 64-lane locomotion teams (Humanoid)
#endif
// and for the hand instances (round 5, same box, profiles/r05/ab_hand_test_solve_width.txt): 12 for the block and
// the pen (ShadowHand 16,384 / 4,096 +1.6 / +2.0 %, pen +1.8 %; 9: +0.4 %, 15: -1 %, 18: -3 to -5 %), 6 for the egg
// (its LDS object rows leave no room: 9 or 12 cost it 18-21 %)
#ifndef MG_RB_HAND
#define MG_RB_HAND 12
#endif
#ifndef MG_RB_EGG
#define MG_RB_EGG 6
#endif

// the tangent basis of a contact normal (stored by build_rows, or recomputed where the compact layout keeps none)
__device__ __forceinline__ void tangent_basis_t(V3 n, V3* t1, V3* t2) {
  V3 a = fabsf(n.x) < 0.57735f ? v3(1, 0, 0) : v3(0, 1, 0);
  V3 t = cross(a, n);
  t = t * prsq(dot(t, t));
  *t1 = t;
  *t2 = cross(n, t);
}

#ifndef MG_PART_B_LDS
#define MG_PART_B_LDS 0  // part-B PGS rows in the dead tree tiles (TeamLDS::PBL); an A/B variant
#endif
template <int T, int MN, int MC, int OBJ = 0>
struct TeamLDS {
  // row capacity, rounded up to a multiple of the PGS prefetch depth (the sweep pads to it)
  static constexpr int MR = (3 * MC + 2 * (MN - 1) + kPgsPrefetch - 1) / kPgsPrefetch * kPgsPrefetch;
  static constexpr int RB = OBJ ? (OBJ == MG_GT_ELLIPSOID ? MG_RB_EGG : MG_RB_HAND) : (T >= 32 ? MG_RB_LOCO32 : (kRBLoco <= T ? kRBLoco : 6));
  // rows whose (J, Y) columns stay in registers during the PGS (a multiple of the prefetch depth)
  // (not for the egg instance: 17.16 vs 17.73 M env-steps/s and 450 vs 409 MB per launch, measured on its fp32 build)
  static constexpr int KR0 = OBJ == MG_GT_ELLIPSOID ? MG_KJY_EGG : (OBJ ? MG_KJY_HAND : (T >= 32 ? MG_KJY_LOCO32 : kJYRegs));
  static constexpr int KR = (KR0 < MR ? KR0 : MR) / kPgsPrefetch * kPgsPrefetch;  // right-hand sides per test solve (rows of 2-4 contacts)
  // part-B rows whose (J, Y) columns live in the LDS left dead by the tree phases (R[1..MN-1], x, V: written by
  // fk(), read by collide(), not again until the next fk()) instead of scratch, one float per lane and row for J
  // and for Y; locomotion instances only (the hand kernels keep their tree tiles live longer: egg_stage /
  // reload_tree, the object rows).  Off by default (MG_PART_B_LDS=1 builds it): same box, it cut Humanoid 32,768's
  // HBM-side traffic 156 -> 119 MB per launch and Ant 65,536's 70.5 -> 61.6 MB, but cost 1.2 % (Humanoid) to 3 %
  // (Ant 16,384, MA-Ant) of throughput (profiles/r05/ab_part_b_lds.txt)
  static constexpr int PBL0 = (OBJ || !MG_PART_B_LDS) ? 0 : (int)(((MN - 1) * 9 + MN * 9) / (2 * T));
  static constexpr int PBL = KR + PBL0 <= MR ? PBL0 : (MR - KR > 0 ? MR - KR : 0);
#if MG_PART_B_LDS
  // S first: the link axes outlive the solve (clamp_ang_vel reads them after the PGS), as does R[0]; the storage
  // from R[1] through V is dead from the end of collide() to the next fk(), and holds part-B PGS rows (PBL)
  float S[MN][6];
  float R[MN][9];
  float x[MN][3];
  float V[MN][6];
#else
  float R[MN][9];
  float x[MN][3];
  float V[MN][6];
  float S[MN][6];
#endif
  float U[MN][6];
  float Dinv[MN];
  float L0[21];
  float Iinv[36];
  int ncon, nrows;
  // contacts: point, frame (normal + tangent basis), gap, sides (nodes / geoms)
  // (hand tasks: once the last substep's outputs have read the contacts, their storage is the
  // observation staging row)
  union {
    struct {
      float cp[MC][3], cn[MC][3], ct1[MC][3], ct2[MC][3];
    };
    float obs[OBJ ? 212 : 1];
  };
  float cd[MC];
  static_assert(!OBJ || 12 * MC >= 212, "the hand's observation row must fit the contact storage");
  int cside[MC];  // packed int8 [node A, node B, geom A, geom B] (-1 none, -2 the free object)
  // joint-limit rows (after the 3 rows per contact): kind | node << 4
  int lmeta[2 * (MN - 1)];
  // The ABA's child slots are dead once its backward pass is done.  The same storage then holds the
  // forward-pass / test-solve accelerations (RB right-hand sides; slab 0 is the ABA's), and behind
  // them the constraint rows: per row {target b, 1/W, impulse, mu (friction: the coefficient; -1 normal, -2 limit)},
  // one 16-byte LDS read.  After the last substep the post-step staging (root row, DOF state, sensor
  // and DOF forces) takes the accelerations' place; the rows region becomes the observation staging
  // once the outputs have read the impulses.
  struct alignas(16) Row { float b, iw, lam, mu; };
  struct Solve {
    union {
      struct {
        float acc[MN][6];  // ABA forward pass
        float proot[6];
      } aba;
      struct {
        float ut[RB][MN];   // test solves: joint-space forces of the RB columns
        float proot[RB][6]; // and their root biases
      } ts;
    };
  };
  struct Stage {
    float root[13];
    float dof[2 * MN];
    float sens[6 * MG_MAX_SENSORS];
    float dforce[MN];
  };
  union {
    float slot[MN][27];
    struct {
      union {
        Solve ts;
        Stage st;
      };
      Row rows[MR];
    } sv;
  } u;
  // free object (OBJ): staged root row, obs staging.  The object part of a contact row, [(p - c) x d; d],
  // is recomputed from the contact list where it is needed (the 2.9 KB per team saved lets 6 blocks
  // share a CU: block 12.5 -> 13.8 M env-steps/s); the egg instance keeps the rows in LDS, whose code
  // the compiler schedules better around the narrowphase (fp64: 5.7 vs 3.6-3.9 M env-steps/s; fp32: 17.73 vs 17.21 M)
  static constexpr int OROWS = OBJ == MG_GT_ELLIPSOID ? 3 * MC : 1;
  float rwo[OROWS][6];
  float oroot[OBJ ? 13 : 1];
  float goal[OBJ ? 26 : 1];   // goal actor root row, goal_states row
  float oforce[OBJ ? 4 : 1];  // external force on the object (apply_rigid_body_force_tensors), [3] = local
  // block / pen: the exact hull candidates of this substep (Team::hull_stage -> collide), world frame
  static constexpr int HX = (OBJ == MG_GT_BOX || OBJ == MG_GT_CAPSULE) ? 2 : 0;
  float hx[HX > 0 ? HX : 1][7];
  int hxn;

  // ---- accessors: the Team reaches every phase-scoped region through these, so the compact layout below (the
  // 16-lane locomotion instances) can place the regions differently
  static constexpr bool kCompact = false;
  static constexpr bool kGwInA = false;
  static constexpr size_t kObsStageBytes = sizeof(Row) * MR;   // the locomotion observation staging (the dead rows)
  static constexpr size_t kGwFloats = (size_t)MN * 27;          // geom frames + pair list + candidate map (collide)
  static constexpr size_t kUtFloats = (size_t)RB * MN;          // the test solves' ut slab (and their y rows)
  __device__ __forceinline__ Row* rows() { return u.sv.rows; }
  __device__ __forceinline__ Stage& st() { return u.sv.st; }
  __device__ __forceinline__ float* qvsc() { return &u.slot[0][0]; }
  __device__ __forceinline__ float* slot(int node, int) { return u.slot[node]; }
  __device__ __forceinline__ float* acc(int node) { return u.sv.ts.aba.acc[node]; }
  __device__ __forceinline__ float* aproot() { return u.sv.ts.aba.proot; }
  __device__ __forceinline__ float* l0() { return L0; }
  __device__ __forceinline__ float* iinv() { return Iinv; }
  __device__ __forceinline__ float* ut(int q) { return u.sv.ts.ts.ut[q]; }
  __device__ __forceinline__ float* tsroot(int q) { return u.sv.ts.ts.proot[q]; }
  __device__ __forceinline__ float* gw() { return &u.slot[0][0]; }
  __device__ __forceinline__ float* obs_stage() { return &u.sv.rows[0].b; }
  __device__ __forceinline__ float gap(int c) const { return cd[c]; }
  __device__ __forceinline__ void set_gap(int c, float d) { cd[c] = d; }
  __device__ __forceinline__ int lm(int i) const { return lmeta[i]; }
  __device__ __forceinline__ void set_lm(int i, int v) { lmeta[i] = v; }
  __device__ __forceinline__ void tangents(int c, V3* t1, V3* t2) const { *t1 = ld3(ct1[c]); *t2 = ld3(ct2[c]); }
  __device__ __forceinline__ void set_tangents(int c, V3 t1, V3 t2) {
    ct1[c][0] = t1.x; ct1[c][1] = t1.y; ct1[c][2] = t1.z;
    ct2[c][0] = t2.x; ct2[c][1] = t2.y; ct2[c][2] = t2.z;
  }
};

// The compact team layout of the 16- and 32-lane locomotion instances (Ant, MA-Ant, Humanoid; MG_COMPACT_LDS,
// common.hpp mg_compact_layout): Ant 4.2 -> 2.8 KB per team, Humanoid 9.0 -> 5.6 KB, so that twelve waves fit a CU's
// 160 KB (three per SIMD) instead of eight.  What it changes against TeamLDS:
//   * region A holds the poses R, x, V from fk() to collide()'s geom staging, then the constraint rows (build_rows()
//     to outputs()), then the observation staging.  The 16-lane layout also keeps each contact's gap in its normal
//     row's b from collide() on; the 32-lane one keeps a gap array and stages collide()'s geom frames in region A
//     instead (read the poses, wave sync, write the frames);
//   * region B holds fk()'s joint sines, the ABA child slots (one per node of a tree level: kCompactLevelSlots, the
//     node's index within its depth from the tile), the ABA forward pass with the root factor and inverse (L0, Iinv:
//     dead once the root coupling Wv is taken, right after aba()), the 16-lane layout's geom frames, the test-solve
//     slab, and after the step the stage rows plus the contacts' impulse sums that outputs() stashes before its fk()
//     overwrites region A;
//   * no tangent basis is stored (recomputed from the normal by tangent_basis_t, the same bits) and the limit-row
//     metadata is one byte per row (two for more than 16 nodes).
// The ancestor masks and the nodes' level slots live in the block's model tile for every instance.
#ifndef MG_HULL_FACE_GROUP
#define MG_HULL_FACE_GROUP 4  // collide(): object points per pass of the hull's face argmax
#endif
#ifndef MG_HULL_PLANE_UNROLL
#define MG_HULL_PLANE_UNROLL 5  // collide(): plane loads in flight per pass of the hull's face argmax
#endif
#ifndef MG_RB_LOCO32C
#define MG_RB_LOCO32C 6   // test-solve columns per batch of the compact 32-lane teams
#endif
#ifndef MG_KJY_LOCO32C
#define MG_KJY_LOCO32C 8  // register rows of (J, Y) of the compact 32-lane teams
#endif
template <int T, int MN, int MC, int MG, int MP>
struct TeamLDSC {
  static_assert(MN <= 32, "the compact limit-row metadata packs the node in 12 bits at most");
  // geom frames (13 floats per geom) and the pair list in region A (and a gap array) for the 32-lane teams and where
  // they do not fit region B's slots; else in region B
  static constexpr bool kGwInA = T >= 32 || MG * 13 + MP > kCompactLevelSlots * 27;
  static constexpr int MR = (3 * MC + 2 * (MN - 1) + kPgsPrefetch - 1) / kPgsPrefetch * kPgsPrefetch;
  static constexpr int RB = T >= 32 ? MG_RB_LOCO32C : (kRBLoco <= T ? kRBLoco : 6);
  static constexpr int KR0 = T >= 32 ? MG_KJY_LOCO32C : kJYRegs;
  static constexpr int KR = (KR0 < MR ? KR0 : MR) / kPgsPrefetch * kPgsPrefetch;
  static constexpr int PBL = 0;
  static constexpr int OROWS = 1;
  static constexpr int HX = 0;
  static constexpr bool kCompact = true;
  using LM = typename std::conditional<(MN <= 16), uint8_t, uint16_t>::type;
  struct alignas(16) Row { float b, iw, lam, mu; };
  struct Stage {
    float root[13];
    float dof[2 * MN];
    float sens[6 * MG_MAX_SENSORS];
    float dforce[MN];
  };
  float S[MN][6];
  float U[MN][6];
  float Dinv[MN];
  int ncon, nrows;
  float cp[MC][3], cn[MC][3];
  int cside[MC];  // packed int8 [node A, node B, geom A, geom B]
  float cd[kGwInA ? MC : 1];
  LM lmeta[(2 * (MN - 1) + 3) / 4 * 4];  // limit rows: kind | node << 4
  union {  // region A
    struct {
      float R[MN][9];
      float x[MN][3];
      float V[MN][6];
    };
    Row rowsA[MR];
  };
  union {  // region B
    float slots[kCompactLevelSlots][27];
    struct {
      float acc[MN][6];
      float proot[6];
      float L0[21];
      float Iinv[36];
    } aba;
    struct {
      float ut[RB][MN];
      float proot[RB][6];
    } ts;
    struct {
      Stage st;
      float fc[MC][3];  // outputs(): each contact's impulse sum n l_n + t1 l_t1 + t2 l_t2
    } post;
    struct {  // the free-object fields of TeamLDS (OBJ = 0 here: never written or read at run time)
      float rwo[1][6];
      float oroot[1], goal[1], oforce[4];
      float hx[1][7];
      int hxn;
      float obs[1];
    };
  };
  static_assert(sizeof(Stage) >= sizeof(float) * 4 * MN, "the stash must lie past fk()'s joint sines");
  static_assert(sizeof(slots) >= sizeof(float) * 4 * MN, "fk()'s joint sines must fit region B");
  static constexpr size_t kRegionA = sizeof(Row) * MR > sizeof(float) * 18 * MN ? sizeof(Row) * MR : sizeof(float) * 18 * MN;
  static constexpr size_t kObsStageBytes = kRegionA;
  static constexpr size_t kGwFloats = kGwInA ? kRegionA / sizeof(float) : (size_t)kCompactLevelSlots * 27;
  static constexpr size_t kUtFloats = (size_t)RB * MN;
  __device__ __forceinline__ Row* rows() { return rowsA; }
  __device__ __forceinline__ Stage& st() { return post.st; }
  __device__ __forceinline__ float* qvsc() { return &slots[0][0]; }
  __device__ __forceinline__ float* slot(int, int lv) { return slots[lv]; }  // by the node's slot in its level
  __device__ __forceinline__ float* acc(int node) { return aba.acc[node]; }
  __device__ __forceinline__ float* aproot() { return aba.proot; }
  __device__ __forceinline__ float* l0() { return aba.L0; }
  __device__ __forceinline__ float* iinv() { return aba.Iinv; }
  __device__ __forceinline__ float* ut(int q) { return ts.ut[q]; }
  __device__ __forceinline__ float* tsroot(int q) { return ts.proot[q]; }
  __device__ __forceinline__ float* gw() { return kGwInA ? &rowsA[0].b : &slots[0][0]; }
  __device__ __forceinline__ float* obs_stage() { return &rowsA[0].b; }
  __device__ __forceinline__ float* fc(int c) { return post.fc[c]; }
  __device__ __forceinline__ float gap(int c) const { return kGwInA ? cd[c] : rowsA[3 * c].b; }
  __device__ __forceinline__ void set_gap(int c, float d) {
    if constexpr (kGwInA) cd[c] = d;
    else rowsA[3 * c].b = d;
  }
  __device__ __forceinline__ int lm(int i) const { return lmeta[i]; }
  __device__ __forceinline__ void set_lm(int i, int v) { lmeta[i] = (LM)v; }
  __device__ __forceinline__ void tangents(int c, V3* t1, V3* t2) const { tangent_basis_t(ld3(cn[c]), t1, t2); }
  __device__ __forceinline__ void set_tangents(int, V3, V3) {}
};
// the team layout of an instance (common.hpp mg_compact_layout)
// LAY: the instance's layout (dispatch.hpp MG_INSTANCES; 1 = compact, for the big batches, where twelve waves per CU pay)
template <int T, int MN, int MC, int OBJ, int MG, int MP, int LAY>
using TeamLDSOf = typename std::conditional<LAY != 0 && mg_compact_layout(T, MN, OBJ), TeamLDSC<T, MN, MC, MG, MP>,
                                            TeamLDS<T, MN, MC, OBJ>>::type;

// A team's LDS region padded so that consecutive teams start 4*T bytes apart modulo 128 B.  A
// ds_read/write_b32 is serviced per 32-lane half with bank = dword address mod 32, so teams of
// T < 32 lanes share a half: without the stagger (Ant's TeamLDS is 3840 B = 30 x 128 B) lane j
// of team 0 and lane j of team 1 hit the same bank on every per-lane or broadcast access
// (measured: SQ_LDS_BANK_CONFLICT ~ 2x SQ_INSTS_LDS for Ant).  With the stagger, per-lane
// accesses at any odd dword stride and team-broadcast reads are conflict-free across the teams.
template <class L, int T, int P = (T < 32) ? (int)((4 * T - (int)(sizeof(L) % 128) + 128) % 128) : 0>
struct alignas(16) BankSlot {
  L v;
  char pad[P];
};
template <class L, int T>
struct alignas(16) BankSlot<L, T, 0> {
  L v;
};

// Per-actor properties under domain randomization (mg_state_views.env_props), one copy per team in
// LDS: nodes [mass, armature, damping, stiffness, lower, upper, drive kp, effort, frictionloss] (rows of 9
// floats, MG_EP_NODE_WIDTH: a node's lane reads its own row, odd stride), geom friction, tendons [limit stiffness, damping],
// object [mass, friction, scale].  The layout of the global row is mg_env_props_layout's.
template <int MN, int MG>
struct DrTile {
  float node[MN][9];
  float geom[MG];
  float ten[MG_MAX_TENDONS][2];
  float obj[4];
};
// copy one env_props row (global) into the team's DrTile, team-cooperative
template <int T, int MN, int MG>
__device__ __forceinline__ void load_dr(DrTile<MN, MG>* d, const float* row, const mg_model* m, int tl) {
  const int nn = m->num_nodes, ng = m->num_geoms, nt = m->num_tendons;
  static_assert(MG_EP_NODE_WIDTH == 9, "DrTile node rows are the global rows");
  for (int k = tl; k < MG_EP_NODE_WIDTH * nn; k += T) (&d->node[0][0])[k] = row[k];
  const float* g = row + MG_EP_NODE_WIDTH * nn;
  for (int k = tl; k < ng; k += T) d->geom[k] = g[k];
  const float* tr = g + ng;
  for (int k = tl; k < 2 * nt; k += T) d->ten[k >> 1][k & 1] = tr[k];
  if (tl < 4) d->obj[tl] = tr[2 * nt + tl];
}

// this team's bits of a 64-lane ballot, at bit 0 (shift the ballot right by the team's first lane)
template <int T>
__device__ __forceinline__ constexpr unsigned long long team_bits() {
  return T >= 64 ? ~0ull : ((1ull << T) - 1ull);
}

// Team reduction with DPP (quad xor 1/2, row_half_mirror, row_mirror) + v_permlane16_swap (xor 16) and
// a bpermute xor 32.  Every step adds a lane to its partner symmetrically, so all lanes of the team
// end with bit-identical sums (fp add is commutative) and no broadcast is needed.
template <int T>
__device__ __forceinline__ float team_sum(float v, int) {
  // no contraction into the butterfly: a lane's product fused into its first add would differ from the
  // rounded product its partner receives, and the team's lanes would no longer hold identical sums
#pragma clang fp contract(off)
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));  // quad xor 1
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));  // quad xor 2
  if (T >= 8) v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));
  if (T >= 16) v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));
  if (T >= 32) {  // xor 16: v_permlane16_swap exchanges the odd 16-lane rows of one copy with the even
                  // rows of the other (gfx950), so the partner value is in the swapped copy
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v += __uint_as_float((threadIdx.x & 16) ? r[0] : r[1]);
  }
  if (T >= 64) v += __shfl_xor(v, 32);
  return v;
}
// the inclusive scan over the team's lanes of 0 <= v < 2^NB (contact-candidate flags and counts) and the team's total: one ballot
// per bit plane, a lane-mask popcount (v_mbcnt) and the plane's bit count, no cross-lane permutes (same-box A/B
// against the permute scan: Humanoid +2.0 %, ShadowHand pen +1.4 %, block +1.0 %, Ant +0.9 %)
template <int T, int NB>
__device__ __forceinline__ int team_scan_bits(int v, int& tot) {
  const int tl = threadIdx.x % T, tb = (threadIdx.x & 63) - tl;
  const unsigned long long tm = (T >= 64 ? ~0ull : ((1ull << T) - 1ull)) << tb;
  int ex = 0;
  tot = 0;
#pragma unroll
  for (int b = 0; b < NB; b++) {
    const unsigned long long bl = __ballot((v >> b) & 1) & tm;
    ex += (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bl >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bl, 0u)) << b;
    tot += __builtin_popcountll(bl) << b;
  }
  return ex + v;
}
// team argmax of (v, i): the largest v, the smallest i among equal v (a serial loop's first maximum)
template <int T>
__device__ __forceinline__ void team_argmax(float& v, int& i) {
  // DPP butterfly (as team_sum): the pair with the larger v, on ties the smaller i, at every step (same-box A/B,
  // with the ballot forms of the wave maxima and the remaining scans: ShadowHand +1.7 %, pen +1.4 %)
  auto step = [&](float ov, int oi) {
    if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
  };
  step(__int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false)),
       __builtin_amdgcn_update_dpp(0, i, 0xB1, 0xF, 0xF, false));
  step(__int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false)),
       __builtin_amdgcn_update_dpp(0, i, 0x4E, 0xF, 0xF, false));
  if (T >= 8)
    step(__int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false)),
         __builtin_amdgcn_update_dpp(0, i, 0x141, 0xF, 0xF, false));
  if (T >= 16)
    step(__int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false)),
         __builtin_amdgcn_update_dpp(0, i, 0x140, 0xF, 0xF, false));
  if (T >= 32) {
    const auto rv = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    const auto ri = __builtin_amdgcn_permlane16_swap((unsigned)i, (unsigned)i, false, false);
    step(__uint_as_float((threadIdx.x & 16) ? rv[0] : rv[1]), (int)((threadIdx.x & 16) ? ri[0] : ri[1]));
  }
  if (T >= 64) step(__shfl_xor(v, 32), __shfl_xor(i, 32));
}
// the wave's maximum of 0 <= v < 2^NB, wave-uniform: a bitwise search with one ballot per bit
static_assert(MG_MAX_HULL_PLANES < 512 && MG_MAX_HULL_VERTS < 512, "candidate counts are scanned in 9 bit planes");
template <int NB>
__device__ __forceinline__ int wave_max_bits(int v) {
  int m = 0;
#pragma unroll
  for (int b = NB - 1; b >= 0; b--) {
    const int c = m | (1 << b);
    if (__ballot(v >= c) != 0ull) m = c;
  }
  return m;
}
template <int T>
__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = max(v, __shfl_xor(v, m));
  return v;
}

constexpr int OBJ_NODE = -2;  // contact side on the free object

// signed distance of point p (box frame) to a box of half extents hb (same rule as the oracle's
// point_box): outside -> distance to the closest point cb, normal away from the box; inside ->
// minus the smallest face depth (ties x, y, z), that face's normal, cb = projection onto it
__device__ __forceinline__ float point_box(V3 p, V3 hb, V3* nb, V3* cb) {
  V3 q = v3(fminf(fmaxf(p.x, -hb.x), hb.x), fminf(fmaxf(p.y, -hb.y), hb.y), fminf(fmaxf(p.z, -hb.z), hb.z));
  if (q.x != p.x || q.y != p.y || q.z != p.z) {
    V3 d = p - q;
    float l = psqrt(dot(d, d));
    *nb = d * prcp(l);
    *cb = q;
    return l;
  }
  // inside: the depth is the nearest face's; the normal blends the faces within kBoxBlend of the nearest one
  // (weight 1 - (depth - nearest) / kBoxBlend), so it turns continuously across the box's medial planes instead
  // of jumping to whichever face fp32 / fp64 rounding makes nearest (oracle point_box, the same rule)
  const float ex0 = hb.x - p.x, ex1 = hb.x + p.x, ey0 = hb.y - p.y, ey1 = hb.y + p.y, ez0 = hb.z - p.z, ez1 = hb.z + p.z;
  const float dm = fminf(fminf(fminf(ex0, ex1), fminf(ey0, ey1)), fminf(ez0, ez1));
  auto wt = [&](float e) { return fmaxf(0.0f, 1.0f - (e - dm) * (1.0f / kBoxBlend)); };
  V3 n = v3(wt(ex0) - wt(ex1), wt(ey0) - wt(ey1), wt(ez0) - wt(ez1));
  const float nl = dot(n, n);
  if (nl < 1e-12f) {  // opposite faces cancel (a thin box entered at its middle): the nearest face, +x +y +z first
    n = dm == ex0 ? v3(1, 0, 0) : dm == ex1 ? v3(-1, 0, 0) : dm == ey0 ? v3(0, 1, 0) : dm == ey1 ? v3(0, -1, 0)
      : dm == ez0 ? v3(0, 0, 1) : v3(0, 0, -1);
  } else {
    n = n * prsq(nl);
  }
  *nb = n;
  *cb = p + n * dm;
  return -dm;
}

// closest parameter of segment a + t u (box frame) to the box (oracle seg_box_t): exact minimum of
// the convex piecewise-quadratic squared distance over the sorted slab crossings; middle of the
// inside portion when the segment passes through the box.  Registers only: a crossing outside (0, 1)
// is replaced by 1 (the segment's end), so the eight breakpoints [0, six crossings, 1] sort with a fixed
// 12-comparator network and the pieces are visited with static indices (the repeated 1s only add empty
// pieces at the end, which the strict comparison never prefers).  The data-dependent count and insertion
// sort of a literal restatement compile to compare / select chains per dynamic index on this target.
__device__ __forceinline__ void seg_box_cx(float& a, float& b) {
  const float lo = fminf(a, b), hi = fmaxf(a, b);
  a = lo;
  b = hi;
}
__device__ __forceinline__ float seg_box_t(V3 a, V3 u, V3 hb, bool* inside) {
  const float av[3] = {a.x, a.y, a.z}, uv[3] = {u.x, u.y, u.z}, hv[3] = {hb.x, hb.y, hb.z};
  float t0 = 0.0f, t1 = 1.0f;
  bool hit = true;
  float bp[8];
  bp[0] = 0.0f;
  bp[7] = 1.0f;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    float ta = 1.0f, tb = 1.0f;
    if (fabsf(uv[k]) < 1e-12f) {
      if (av[k] < -hv[k] || av[k] > hv[k]) hit = false;
    } else {
      const float iu = prcp(uv[k]);
      ta = (-hv[k] - av[k]) * iu;
      tb = (hv[k] - av[k]) * iu;
      t0 = fmaxf(t0, fminf(ta, tb));
      t1 = fminf(t1, fmaxf(ta, tb));
    }
    bp[1 + 2 * k] = (ta > 0.0f && ta < 1.0f) ? ta : 1.0f;
    bp[2 + 2 * k] = (tb > 0.0f && tb < 1.0f) ? tb : 1.0f;
  }
  *inside = hit && t0 <= t1;
  if (*inside) return 0.5f * (t0 + t1);
  float* c = bp + 1;  // the six crossings
  seg_box_cx(c[0], c[5]); seg_box_cx(c[1], c[3]); seg_box_cx(c[2], c[4]);
  seg_box_cx(c[1], c[2]); seg_box_cx(c[3], c[4]);
  seg_box_cx(c[0], c[3]); seg_box_cx(c[2], c[5]);
  seg_box_cx(c[0], c[1]); seg_box_cx(c[2], c[3]); seg_box_cx(c[4], c[5]);
  seg_box_cx(c[1], c[2]); seg_box_cx(c[3], c[4]);
  float best_t = 0.0f, best_f = 3.0e38f;
#pragma unroll
  for (int i = 0; i < 7; i++) {
    const float lo = bp[i], hi = bp[i + 1], mid = 0.5f * (lo + hi);
    float num = 0.0f, den = 0.0f;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const float x = av[k] + mid * uv[k];
      if (x > hv[k]) { num += (av[k] - hv[k]) * uv[k]; den += uv[k] * uv[k]; }
      else if (x < -hv[k]) { num += (av[k] + hv[k]) * uv[k]; den += uv[k] * uv[k]; }
    }
    float t = den > 0.0f ? -num * prcp(den) : lo;
    t = fminf(fmaxf(t, lo), hi);
    float f = 0.0f;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const float x = fabsf(av[k] + t * uv[k]) - hv[k];
      if (x > 0.0f) f += x * x;
    }
    if (f < best_f) { best_f = f; best_t = t; }
  }
  return best_t;
}

// A segment a + t u whose core has entered a box (seg_box_t's inside case; oracle seg_box_sat): the face of least
// push-out of the whole segment -- SAT over the box's face axes, delta(k, s) = hb_k - min(s a_k, s (a_k + u_k)),
// ties in x+ x- y+ y- z+ z- order -- and the segment end deepest behind it (*t = 0 or 1).  The inside portion's
// midpoint lies on a thin box's mid-plane by construction when the segment pierces it (the reference's pen reset
// pose through the palm), where fp32 and fp64 picked opposite faces; the whole segment's extents decide robustly.
__device__ __forceinline__ int seg_box_sat(V3 a, V3 u, V3 hb, float* t) {
  const float av[3] = {a.x, a.y, a.z}, ev[3] = {a.x + u.x, a.y + u.y, a.z + u.z}, hv[3] = {hb.x, hb.y, hb.z};
  int best = 0;
  float bd = 3.0e38f;
#pragma unroll
  for (int f = 0; f < 6; f++) {
    const int k = f >> 1;
    const float sg = (f & 1) ? -1.0f : 1.0f;
    const float dl = hv[k] - fminf(sg * av[k], sg * ev[k]);
    if (dl < bd) { bd = dl; best = f; }
  }
  const int k = best >> 1;
  const float sg = (best & 1) ? -1.0f : 1.0f;
  const float a0 = k == 0 ? a.x : (k == 1 ? a.y : a.z), a1 = k == 0 ? ev[0] : (k == 1 ? ev[1] : ev[2]);
  *t = sg * a0 <= sg * a1 ? 0.0f : 1.0f;
  return best;
}
// signed distance of P (box frame) along face f's outward normal from that face's plane (negative behind it);
// nb = the normal, cb = P moved onto the plane (oracle box_face_point)
__device__ __forceinline__ float box_face_point(V3 P, V3 hb, int f, V3* nb, V3* cb) {
  const int k = f >> 1;
  const float sg = (f & 1) ? -1.0f : 1.0f;
  *nb = v3(k == 0 ? sg : 0.0f, k == 1 ? sg : 0.0f, k == 2 ? sg : 0.0f);
  const float pk = k == 0 ? P.x : (k == 1 ? P.y : P.z), hk = k == 0 ? hb.x : (k == 1 ? hb.y : hb.z);
  *cb = v3(k == 0 ? sg * hk : P.x, k == 1 ? sg * hk : P.y, k == 2 ? sg * hk : P.z);
  return sg * pk - hk;
}
// the segment's contact point against a box (P, box frame) with its normal / surface point: the closest point
// outside, the seg_box_sat face inside; returns the signed distance of the core
__device__ __forceinline__ float seg_box_point(V3 a, V3 u, V3 hb, V3* P, V3* nb, V3* cb) {
  bool inside;
  float t = seg_box_t(a, u, hb, &inside);
  if (inside) {
    const int f = seg_box_sat(a, u, hb, &t);
    *P = a + u * t;
    return box_face_point(*P, hb, f, nb, cb);
  }
  *P = a + u * t;
  return point_box(*P, hb, nb, cb);
}

// ---- the convex-mesh geom (MG_GT_CONVEX; oracle point_hull / hull_box_near): the model's hull tables are read
// from global memory (only the few candidates near the hull touch them)
// largest plane distance of pl (geom frame) over the hull's faces (*f = the face): the signed distance inside
// and where a face is the nearest feature, a lower bound outside near edges / vertices
__device__ __forceinline__ float point_hull(const mg_model* m, V3 pl, int* f) {
  float best = -3.0e38f;
  int bf = 0;
  const int np = m->hull_num_planes;
  for (int i = 0; i < np; i++) {
    const float* q = m->hull_plane[i];
    const float sd = q[0] * pl.x + q[1] * pl.y + q[2] * pl.z - q[3];
    if (sd > best) { best = sd; bf = i; }
  }
  *f = bf;
  return best;
}
// the hull's bounding box (half extents hg about the geom centre c, axes Rg) within off of a sphere (w, r)
__device__ __forceinline__ bool hull_box_near(V3 c, const M3& Rg, V3 hg, V3 w, float r, float off) {
  const V3 l = mulT(Rg, w - c);
  const float ex = fmaxf(fabsf(l.x) - hg.x, 0.0f), ey = fmaxf(fabsf(l.y) - hg.y, 0.0f), ez = fmaxf(fabsf(l.z) - hg.z, 0.0f);
  return psqrt(ex * ex + ey * ey + ez * ez) - r < off;
}

// box-box edge-edge contact in the object box's frame (oracle box_box_edge): hand box centre c, axes = the
// columns of R, half extents hg; object half extents hb.  SAT over the 15 axes (edge axes within ~11 deg of a
// face normal left to the face contacts); an edge axis better than every face axis by 1e-5 m with a
// separation below off gives one contact at the supporting edges' closest points, normal from B to A.
__device__ __forceinline__ bool box_box_edge(V3 c, const M3& R, V3 hg, V3 hb, float off, V3* pt, V3* nrm, float* dist) {
  const float cv[3] = {c.x, c.y, c.z}, hgv[3] = {hg.x, hg.y, hg.z}, hbv[3] = {hb.x, hb.y, hb.z};
  float face = -3.0e38f;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const float ra = hgv[0] * fabsf(R.m[i][0]) + hgv[1] * fabsf(R.m[i][1]) + hgv[2] * fabsf(R.m[i][2]);
    face = fmaxf(face, fabsf(cv[i]) - hbv[i] - ra);
  }
#pragma unroll
  for (int j = 0; j < 3; j++) {
    const float t = R.m[0][j] * cv[0] + R.m[1][j] * cv[1] + R.m[2][j] * cv[2];
    const float rb = hbv[0] * fabsf(R.m[0][j]) + hbv[1] * fabsf(R.m[1][j]) + hbv[2] * fabsf(R.m[2][j]);
    face = fmaxf(face, fabsf(t) - hgv[j] - rb);
  }
  // edge axes e_i x a_j in closed form from the entries of R (oracle box_box_edge)
  float best = -3.0e38f;
  int bi = -1, bj = -1;
  float L[3] = {0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) {
      const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
      const float ln = psqrt(R.m[i1][j] * R.m[i1][j] + R.m[i2][j] * R.m[i2][j]);
      if (ln < 1e-6f) continue;
      const float il = prcp(ln);
      const float near = fmaxf(fmaxf(fabsf(R.m[i1][j]), fabsf(R.m[i2][j])), fmaxf(fabsf(R.m[i][j1]), fabsf(R.m[i][j2]))) * il;
      if (near > 0.98f) continue;
      const float tl = cv[i2] * R.m[i1][j] - cv[i1] * R.m[i2][j];
      const float rb = hbv[i1] * fabsf(R.m[i2][j]) + hbv[i2] * fabsf(R.m[i1][j]);
      const float ra = hgv[j1] * fabsf(R.m[i][j2]) + hgv[j2] * fabsf(R.m[i][j1]);
      const float sep = (fabsf(tl) - ra - rb) * il;
      if (sep > best) {
        const float sg = tl < 0.0f ? -1.0f : 1.0f;
        best = sep; bi = i; bj = j;
        L[i] = 0.0f;
        L[i1] = -sg * R.m[i2][j] / ln;
        L[i2] = sg * R.m[i1][j] / ln;
      }
    }
  if (bi < 0 || !(best > face + 1e-5f) || !(best < off)) return false;
  // the supporting edges (B: parallel to e_bi, the corner towards +L; A: parallel to a_bj, towards -L);
  // bi / bj are data dependent, so columns and extents are selected by unrolled compares (no dynamic
  // register indexing, which would put R in scratch)
  float pb[3], pa[3] = {cv[0], cv[1], cv[2]}, hga = 0.0f, hbb = 0.0f;
  V3 ua = v3(0, 0, 0);
#pragma unroll
  for (int a = 0; a < 3; a++) {
    pb[a] = a == bi ? 0.0f : (L[a] >= 0.0f ? hbv[a] : -hbv[a]);
    if (a == bi) hbb = hbv[a];
  }
#pragma unroll
  for (int k = 0; k < 3; k++) {
    if (k == bj) {
      ua = v3(R.m[0][k], R.m[1][k], R.m[2][k]);
      hga = hgv[k];
      continue;
    }
    const float sg = (L[0] * R.m[0][k] + L[1] * R.m[1][k] + L[2] * R.m[2][k]) >= 0.0f ? -hgv[k] : hgv[k];
#pragma unroll
    for (int a = 0; a < 3; a++) pa[a] += sg * R.m[a][k];
  }
  const V3 ub = v3(bi == 0 ? 1.0f : 0.0f, bi == 1 ? 1.0f : 0.0f, bi == 2 ? 1.0f : 0.0f);
  const V3 PA = v3(pa[0], pa[1], pa[2]), PB = v3(pb[0], pb[1], pb[2]), w0 = PA - PB;
  const float b = dot(ua, ub), dd = dot(ua, w0), e = dot(ub, w0), den = 1.0f - b * b;
  if (den < 1e-12f) return false;
  const float iden = prcp(den);
  const float sa = (b * e - dd) * iden, tb = (e - b * dd) * iden;
  if (fabsf(sa) > hga || fabsf(tb) > hbb) return false;
  *pt = ((PA + ua * sa) + (PB + ub * tb)) * 0.5f;
  *nrm = v3(L[0], L[1], L[2]);
  *dist = best;
  return true;
}

// Per-lane context of one team.  Every member function is force-inlined: one that the inliner leaves as a
// call (it declined fk() once the egg kernel grew) takes `this`, which puts the whole Team object in scratch
// memory, and every phase then runs from scratch (egg: 7.4 -> 4.7 M env-steps/s until this was found).
// OBJ: the free object's type (0: none); TGS: the build's TGS solver (mg_sim_params.solver_type) -- its
// own kernel instances, so the PGS instances are the code they were
template <int T, int MN, int MC, int MG, int MP, int OBJ = 0, bool TGS = false, int LAY = 0>
struct Team {
  using L = TeamLDSOf<T, MN, MC, OBJ, MG, MP, LAY>;
  using MT = ModelTile<MN, MG, MP, tile_hull_verts(OBJ)>;
  static constexpr int MR = L::MR;
#ifndef MG_HW_TRIG_T16
#define MG_HW_TRIG_T16 1
#endif
#ifndef MG_SENSOR_MASKS
#define MG_SENSOR_MASKS 1  // outputs(): per-sensor contact masks by ballots instead of every sensor scanning every contact
#endif
#ifndef MG_LOAD_RSQ
#define MG_LOAD_RSQ 1  // load(): free-base root quaternions normalised by rsq
#endif
  // the hardware sine / cosine for the 16-lane teams (Ant, MA-Ant), the library's elsewhere (device_math.hpp psincos)
  static constexpr bool kHwTrig = MG_HW_TRIG_T16 && T == 16 && OBJ == 0;
  L* s;
  const MT* mt;
  const mg_model* m;
  const mg_sim_params* p;
  int tl, tb;          // team lane, first lane of the team within its wave
  bool freeb;
  int nn, nv, ncol0;   // nodes, velocity columns, first joint column
  int node;            // node owned by this lane (-1: none)
  int depth, maxdepth;
  int par;
  // state
  float nu;            // generalized velocity column tl (valid if tl < nv)
  float qj, tau;       // joint position / actuation (node lanes)
  V3 p0;               // root position (lane 0)
  float q0[4];         // root orientation (lane 0)
  // kinematics / dynamics of own node
  M3 R;
  V3 x;
  SV S, V, c, U, pA;
  Sym6 IA;
  float Dinv, u;
  float h;
  float Sl[6];         // Jacobian axis of the lane: S (joint lanes) or e_tl (root-twist lanes)
  int ncr;             // contacts of this substep (rows 0 .. 3 ncr - 1 are contact rows)
  V3 org;              // team origin o (root position at the start of the substep)
#ifdef MG_PHASE_TIMING
  // shader-clock cycles per solver phase (profiling build only, see build.py --timing); wave-uniform
  // 32-bit accumulators so they stay in SGPRs and do not disturb the vector register budget
  unsigned int ph[MG_NUM_PHASES];
  unsigned long long tmark;
  __device__ __forceinline__ void ph_start() {
    for (int i = 0; i < MG_NUM_PHASES; i++) ph[i] = 0u;
    tmark = __builtin_amdgcn_s_memtime();
  }
  __device__ __forceinline__ void ph_mark(int i) {
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    ph[i] = __builtin_amdgcn_readfirstlane(ph[i] + (unsigned int)(t1 - tmark));
    tmark = t1;
  }
#else
  __device__ __forceinline__ void ph_start() {}
  __device__ __forceinline__ void ph_mark(int) {}
#endif
  // drives / tendons (node lanes)
  float tgt;           // PD target of the own DOF
  float ttend;         // tendon generalized force (current substep)
  int sat;             // bit 0: drive saturated (current substep); bits 1 / 2: a lower / upper limit row, bits 3+: its
                       // index among the limit rows (build_rows; outputs() reads the DOF force's limit impulses there)
  // domain randomization: the team's DrTile (nullptr: the model's constants)
  const float* drn;    // node rows (stride 9)
  const float* drg;    // geom friction
  const float* drt;    // tendons (stride 2)
  const float* dro;    // object [mass, friction, scale]
  // node property row [mass, armature, damping, stiffness, lower, upper, drive kp, effort, frictionloss]: the DR row
  // or the tile's nf[24..32]
  __device__ __forceinline__ const float* nprop(int i) const { return drn ? drn + MG_EP_NODE_WIDTH * i : &mt->nf[i][24]; }
  __device__ __forceinline__ float omass() const { return dro ? dro[0] : m->obj_mass; }
  __device__ __forceinline__ float oscale() const { return dro ? dro[2] : 1.0f; }
  __device__ __forceinline__ V3 osize() const { return ld3(m->obj_size) * oscale(); }
  // object principal moments: model inertia x (mass / model mass) x scale^2 (uniform density)
  __device__ __forceinline__ V3 oinertia() const {
    const float f = dro ? (dro[0] / m->obj_mass) * dro[2] * dro[2] : 1.0f;
    return ld3(m->obj_inertia) * f;
  }
  // friction coefficient of a contact side's geom (-1 ground plane, -2 the object)
  __device__ __forceinline__ float gmu(int g) const { return g >= 0 ? drg[g] : (g == -2 ? dro[1] : p->friction); }
  // free object (OBJ): pose replicated on every lane, velocity column on lanes ob0..ob0+5
  int ob0;
  bool objl;
  V3 op;
  float oq[4];
  M3 oR;

  __device__ __forceinline__ int col_of(int i) const { return ncol0 - 1 + i; }

  __device__ __forceinline__ void init(L* lds, const MT* tile, const mg_model* mm, const mg_sim_params* pp,
                                       bool opaque_lane = false) {
    s = lds;
    mt = tile;
    m = mm;
    p = pp;
    drn = drg = drt = dro = nullptr;
    tl = threadIdx.x % T;
    // opaque_lane: tl made opaque to the optimizer.  The work-queue step kernels call init() once per work
    // item, and every lane-dependent constant derived from tl would otherwise be hoisted out of their work
    // loop and held in registers across it
    if (opaque_lane) asm volatile("" : "+v"(tl));
    tb = (threadIdx.x & 63) - tl;  // first lane of the team within its wave
    freeb = !m->fixed_base;
    nn = m->num_nodes;
    ncol0 = freeb ? 6 : 0;
    nv = ncol0 + nn - 1;
    node = -1;
    if (freeb && tl == 0) node = 0;
    if (tl >= ncol0 && tl - ncol0 + 1 < nn) node = tl - ncol0 + 1;
    par = node > 0 ? mt->parent[node] : -1;
    depth = 0;
    if (node > 0)
      for (int k = node; k > 0; k = mt->parent[k]) depth++;
    maxdepth = wave_max<T>(depth);
    h = p->dt / (float)p->substeps;
    nu = 0.0f;
    qj = 0.0f;
    tau = 0.0f;
    tgt = 0.0f;
    ttend = 0.0f;
    sat = 0;
    ob0 = nv;
    objl = OBJ && tl >= nv && tl < nv + 6;
    op = v3(0, 0, 0);
    oq[0] = oq[1] = oq[2] = 0.0f;
    oq[3] = 1.0f;
  }
  __device__ __forceinline__ float gscale() const { return m->gravity_off ? 0.0f : 1.0f; }
  __device__ __forceinline__ bool in_path(int target, int k) const { return target >= 0 && ((mt->anc[target] >> k) & 1ull); }

  // ---------------------------------------------------------------- FK (level-synchronous)
  // Forward kinematics without a barrier per tree level: every node's lane composes its own path from the
  // root (proper ancestors in increasing depth = increasing index, then itself) with the ancestors' joint
  // positions / velocities published once in LDS.  The operations per link are those of a level-by-level pass
  // (R = R_parent R_rest rot(axis, q), x, S, V = V_parent + S qd), so the results are bit-identical to it; the
  // deeper lanes repeat their ancestors' few dozen FMAs instead of waiting for one LDS round trip and wave
  // barrier per level.  R, x, V, S are then stored for the later phases.  POSE: R and x only (the post-step
  // sensor frames of the fused locomotion step, which reads no velocity or axis after it; R and x are computed
  // by the same operations either way)
  template <bool POSE = false>
  __device__ __forceinline__ void fk() {
    MG_NC_FK
    if (OBJ) oR = quat_to_mat(oq[0], oq[1], oq[2], oq[3]);
    const M3 Rr = quat_to_mat(q0[0], q0[1], q0[2], q0[3]);
    if (tl == 0) {
      for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) s->R[0][3 * a + b] = Rr.m[a][b];
      s->x[0][0] = p0.x; s->x[0][1] = p0.y; s->x[0][2] = p0.z;
      if (!freeb && !POSE)
        for (int k = 0; k < 6; k++) s->V[0][k] = 0.0f;
    }
    if (freeb && tl < 6 && !POSE) s->V[0][tl] = nu;
    // (q, qd) and (sin q, cos q) per node in the union storage (free here: the ABA's child slots are written
    // after): each lane evaluates its own joint's sine and cosine once, its descendants read them
    float* qv = s->qvsc();
    float* sc = qv + 2 * MN;
    static_assert(L::kGwFloats >= 4 * MN, "joint states must fit the union storage");
    float sn = 0.0f, cs = 1.0f;
    if (node > 0) {
      qv[2 * node] = qj;
      qv[2 * node + 1] = nu;
      if (mt->jtype[node] == MG_JT_HINGE) {
        psincos<kHwTrig>(qj, &sn, &cs);
      }
      sc[2 * node] = sn;
      sc[2 * node + 1] = cs;
    }
    wsync();
    if (node >= 0) {
      for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) R.m[a][b] = s->R[0][3 * a + b];
      x = ld3(s->x[0]);
      if (!POSE) V = sv(ld3(s->V[0]), ld3(s->V[0] + 3));
    }
    if (node > 0) {
      const V3 x0 = x;
      for (unsigned long long path = mt->anc[node] & ~1ull; path; path &= path - 1) {
        const int k = __builtin_ctzll(path);
        const float* nf = mt->nf[k];
        M3 R0;
        for (int a = 0; a < 3; a++)
          for (int b = 0; b < 3; b++) R0.m[a][b] = nf[3 * a + b];
        const M3 Rp0 = mul(R, R0);
        const V3 tp = mul(R, ld3(nf + 9));
        const V3 ax = ld3(nf + 12);
        const float qk = k == node ? qj : qv[2 * k], vk = k == node ? nu : qv[2 * k + 1];
        if (mt->jtype[k] == MG_JT_HINGE) {
          R = mul(Rp0, axis_angle_sc(ax, k == node ? sn : sc[2 * k], k == node ? cs : sc[2 * k + 1]));
          x = x + tp;
          if (!POSE) {
            const V3 sw = mul(R, ax);
            S = sv(sw, cross(x - x0, sw));
          }
        } else {
          R = Rp0;
          const V3 sw = mul(Rp0, ax);
          x = x + tp + sw * qk;
          if (!POSE) S = sv(v3(0, 0, 0), sw);
        }
        if (!POSE) V = V + S * vk;
      }
      for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) s->R[node][3 * a + b] = R.m[a][b];
      s->x[node][0] = x.x; s->x[node][1] = x.y; s->x[node][2] = x.z;
      if (!POSE) {
        s->V[node][0] = V.a.x; s->V[node][1] = V.a.y; s->V[node][2] = V.a.z;
        s->V[node][3] = V.l.x; s->V[node][4] = V.l.y; s->V[node][5] = V.l.z;
        s->S[node][0] = S.a.x; s->S[node][1] = S.a.y; s->S[node][2] = S.a.z;
        s->S[node][3] = S.l.x; s->S[node][4] = S.l.y; s->S[node][5] = S.l.z;
      }
    }
    wsync();
  }

  __device__ __forceinline__ void set_axis() {
    if (freeb && tl < 6) {
      for (int k = 0; k < 6; k++) Sl[k] = k == tl ? 1.0f : 0.0f;
    } else {
      Sl[0] = S.a.x; Sl[1] = S.a.y; Sl[2] = S.a.z; Sl[3] = S.l.x; Sl[4] = S.l.y; Sl[5] = S.l.z;
    }
  }

  // ---------------------------------------------------------------- ABA (unconstrained step)
  __device__ __forceinline__ void aba() {
    MG_NC_ABA
    if (node >= 0) {
      const V3 o = ld3(s->x[0]);
      const float* nf = mt->nf[node];
      V3 cc = x + mul(R, ld3(nf + 15)) - o;
      const float* in = nf + 18;
      const float isc = (drn && nf[24] > 0.0f) ? drn[MG_EP_NODE_WIDTH * node] / nf[24] : 1.0f;  // DR: inertia scales with the body mass
      float Il[3][3] = {{in[0] * isc, in[3] * isc, in[4] * isc}, {in[3] * isc, in[1] * isc, in[5] * isc},
                        {in[4] * isc, in[5] * isc, in[2] * isc}};
      float Tm[3][3], Iw[6];
      for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) Tm[a][b] = R.m[a][0] * Il[0][b] + R.m[a][1] * Il[1][b] + R.m[a][2] * Il[2][b];
      const int idx[6][2] = {{0, 0}, {0, 1}, {0, 2}, {1, 1}, {1, 2}, {2, 2}};
      for (int k = 0; k < 6; k++) {
        int a = idx[k][0], b = idx[k][1];
        Iw[k] = Tm[a][0] * R.m[b][0] + Tm[a][1] * R.m[b][1] + Tm[a][2] * R.m[b][2];
      }
      const float mass = drn ? drn[MG_EP_NODE_WIDTH * node] : nf[24];
      IA = body_inertia(mass, cc, Iw);
      SV IV = mul(IA, V);
      V3 mg = ld3(p->gravity) * (mass * gscale());
      pA = crf(V, IV) - sv(cross(cc, mg), mg);
      // link angular damping (gym AssetOptions.angular_damping, mg_model.link_ang_damping): the couple
      // -c I_w w, implicit: + c I_w w in the bias, + h c I_w in the link's rotational block, so a free
      // link's w decays by 1/(1 + h c) per substep and the test solves see the same M~
      const float cd = m->link_ang_damping;
      if (cd != 0.0f) {
        pA.a = pA.a + symmul(Iw, V.a) * cd;
        const float hcd = h * cd;
        for (int k = 0; k < 6; k++) IA.a[k] += hcd * Iw[k];
      }
      c = node == 0 ? szero() : crm(V, S * nu);
    }
    // the joint's own terms of D and u (they do not depend on the subtree), once per lane before the level loop
    // (same-box A/B against computing them inside the level loop: Humanoid +1.1 %, Ant +0.4 %)
    float Dj = 0.0f, tj = 0.0f;
    if (node > 0) {
      const float* np = nprop(node);  // [mass, arm, damp, stiff, lower, upper, kp, effort]
      // implicit spring/damper; PD drives toward the target unless the explicit estimate
      // exceeds the effort limit (then a constant +-limit force, no implicit terms)
      float kk = np[3], bb = np[2], ref = 0.0f, tadd = 0.0f;
      sat = 0;
      if (np[6] > 0.0f) {
        const float fe = np[6] * (tgt - qj) - np[2] * nu;
        if (fabsf(fe) > np[7]) {
          kk = 0.0f; bb = 0.0f; tadd = fe > 0.0f ? np[7] : -np[7]; sat = 1;
        } else {
          kk = np[6]; ref = tgt;
        }
      }
      Dj = np[1] + h * bb + h * h * kk;
      tj = tau + tadd + ttend - bb * nu - kk * (qj - ref + h * nu);
      // dry joint friction (MJCF frictionloss; domain randomization of dof_properties.friction scales this torque
      // bound, column 8 of the DR node row -- not a PhysX-style friction coefficient): -f tanh(qd / v_s), linearly implicit
#ifndef MG_NO_FRICTIONLOSS  // (A/B builds only)
      const float fl = np[8];  // nf[32] or the DR row's
#else
      const float fl = 0.0f;
#endif
      if (fl > 0.0f) {
        const float th = ptanh(nu * (1.0f / MG_FRICTIONLOSS_VS));
        tj -= fl * th;
        Dj += h * fl * (1.0f / MG_FRICTIONLOSS_VS) * (1.0f - th * th);
      }
    }
    ph_mark(16);
    for (int lev = maxdepth; lev >= 1; lev--) {
      // compact layout: the slots are per level, so this level's writes reuse the slots the previous level's parents
      // read just before (a wave's LDS operations complete in order; the sync keeps the compiler from moving them)
      if constexpr (L::kCompact) wsync();
      if (node > 0 && depth == lev) {
        U = mul(IA, S);
        Dinv = prcp(dot(S, U) + Dj);
        u = tj - dot(S, pA);
        Sym6 Ia = IA;
        rank1_sub(Ia, U, Dinv);
        SV pa = pA + mul(Ia, c) + U * (u * Dinv);
        float* sl = s->slot(node, mt->lvs[node]);
        for (int k = 0; k < 6; k++) { sl[k] = Ia.a[k]; sl[15 + k] = Ia.c[k]; }
        for (int k = 0; k < 9; k++) sl[6 + k] = Ia.b[k];
        sl[21] = pa.a.x; sl[22] = pa.a.y; sl[23] = pa.a.z;
        sl[24] = pa.l.x; sl[25] = pa.l.y; sl[26] = pa.l.z;
        s->U[node][0] = U.a.x; s->U[node][1] = U.a.y; s->U[node][2] = U.a.z;
        s->U[node][3] = U.l.x; s->U[node][4] = U.l.y; s->U[node][5] = U.l.z;
        s->Dinv[node] = Dinv;
      }
      wsync();
      if (node >= 0 && depth == lev - 1) {
        unsigned long long ch = mt->children[node];
        while (ch) {
          const int k = __builtin_ctzll(ch);
          ch &= ch - 1;
          const float* sl = s->slot(k, mt->lvs[k]);
          for (int q = 0; q < 6; q++) { IA.a[q] += sl[q]; IA.c[q] += sl[15 + q]; }
          for (int q = 0; q < 9; q++) IA.b[q] += sl[6 + q];
          pA = pA + sv(v3(sl[21], sl[22], sl[23]), v3(sl[24], sl[25], sl[26]));
        }
      }
    }
    ph_mark(17);
    if (tl == 0) {
      if (freeb) {
        chol6(IA, s->l0());
        s->aproot()[0] = pA.a.x; s->aproot()[1] = pA.a.y; s->aproot()[2] = pA.a.z;
        s->aproot()[3] = pA.l.x; s->aproot()[4] = pA.l.y; s->aproot()[5] = pA.l.z;
      } else {
        for (int k = 0; k < 6; k++) s->acc(0)[k] = 0.0f;
      }
    }
    wsync();
    if (freeb && tl < 6) {
      // column tl of IA0^-1 from the Cholesky factor (6 lanes in parallel); a0 = -IA0^-1 pA0
      const SV e = sv(v3(tl == 0 ? 1.f : 0.f, tl == 1 ? 1.f : 0.f, tl == 2 ? 1.f : 0.f),
                      v3(tl == 3 ? 1.f : 0.f, tl == 4 ? 1.f : 0.f, tl == 5 ? 1.f : 0.f));
      SV col = chol6_solve(s->l0(), e);
      float cv[6] = {col.a.x, col.a.y, col.a.z, col.l.x, col.l.y, col.l.z};
      float a = 0.0f;
      for (int k = 0; k < 6; k++) {
        s->iinv()[6 * k + tl] = cv[k];
        a -= cv[k] * s->aproot()[k];
      }
      s->acc(0)[tl] = a;
    }
    wsync();
    ph_mark(18);
    float qdd = 0.0f;
    for (int lev = 1; lev <= maxdepth; lev++) {
      if (node > 0 && depth == lev) {
        SV ap = sv(ld3(s->acc(par)), ld3(s->acc(par) + 3)) + c;
        qdd = (u - dot(U, ap)) * Dinv;
        SV a = ap + S * qdd;
        s->acc(node)[0] = a.a.x; s->acc(node)[1] = a.a.y; s->acc(node)[2] = a.a.z;
        s->acc(node)[3] = a.l.x; s->acc(node)[4] = a.l.y; s->acc(node)[5] = a.l.z;
      }
      wsync();
    }
    // nu* = nu + h * acc
    if (tl < nv) {
      float a = (freeb && tl < 6) ? s->acc(0)[tl] : qdd;
      nu += h * a;
    }
  }

  // ---------------------------------------------------------------- fixed tendons (explicit soft limits)
  __device__ __forceinline__ void tendons() {
    ttend = 0.0f;
    for (int q = 0; q < mt->nten; q++) {
      const int d0 = mt->tdof[q][0], d1 = mt->tdof[q][1];
      const int l0 = tb + ncol0 + d0, l1 = tb + ncol0 + d1;
      const float q0 = __shfl(qj, l0), q1 = __shfl(qj, l1), v0 = __shfl(nu, l0), v1 = __shfl(nu, l1);
      const float* f = mt->tf[q];
      const float Lt = f[0] * q0 + f[1] * q1, Ld = f[0] * v0 + f[1] * v1;
      const float cl = fminf(fmaxf(Lt, f[2]), f[3]);
      const float kl = drt ? drt[2 * q] : f[4], bd = drt ? drt[2 * q + 1] : f[5];
      const float F = -kl * (Lt - cl) - bd * Ld;
      if (node > 0 && node - 1 == d0) ttend += f[0] * F;
      if (node > 0 && node - 1 == d1) ttend += f[1] * F;
    }
  }

  // ---------------------------------------------------------------- free object: unconstrained step
  // I_w = R diag(I) R^T; every lane evaluates the 3-vectors, object lane k keeps component k.
  __device__ __forceinline__ V3 obj_inv_inertia(V3 x) const {
    const V3 I = oinertia();
    V3 b = mulT(oR, x);
    return mul(oR, v3(b.x * prcp(I.x), b.y * prcp(I.y), b.z * prcp(I.z)));  // 1-ulp reciprocals, as the physics
  }
  __device__ __forceinline__ void obj_free() {
    if (!OBJ) return;
    const V3 w = v3(__shfl(nu, tb + ob0), __shfl(nu, tb + ob0 + 1), __shfl(nu, tb + ob0 + 2));
    const V3 I = oinertia();
    const V3 b = mulT(oR, w);
    const V3 Iw = mul(oR, v3(I.x * b.x, I.y * b.y, I.z * b.z));
    const V3 aw = obj_inv_inertia(cross(w, Iw) * -1.0f);
    if (objl) {
      const int k = tl - ob0;
      // applied force at the COM (LOCAL_SPACE: rotated by the orientation at the start of the substep)
      const V3 fl = v3(s->oforce[0], s->oforce[1], s->oforce[2]);
      const V3 fw = s->oforce[3] != 0.0f ? mul(oR, fl) : fl;
      const float fk = k == 3 ? fw.x : k == 4 ? fw.y : fw.z;
      const float a = k == 0 ? aw.x : k == 1 ? aw.y : k == 2 ? aw.z : m->obj_gravity * p->gravity[k - 3] + fk / omass();
      nu += h * a;
      nu *= k < 3 ? 1.0f / (1.0f + h * m->obj_ang_damping) : 1.0f / (1.0f + h * m->obj_lin_damping);
    }
  }
  // object part of contact row r on the object's columns [w; v_com]: +-[(p - c_obj) x d; d] (d = the
  // row's direction: normal or a tangent; sign + when the object is side A)
  __device__ __forceinline__ void obj_jrow(int r, V3* wo, V3* d) const {
    const int c = r / 3, q = r - 3 * c;
    const float so = (cside(c, 0) == OBJ_NODE ? 1.0f : 0.0f) - (cside(c, 1) == OBJ_NODE ? 1.0f : 0.0f);
    V3 t1, t2;
    s->tangents(c, &t1, &t2);
    const V3 dir = q == 0 ? ld3(s->cn[c]) : (q == 1 ? t1 : t2);
    *wo = cross(ld3(s->cp[c]) - op, dir) * so;
    *d = dir * so;
  }
  // object part of the response column Y_r = M^-1 J_r^T (object lanes)
  __device__ __forceinline__ float obj_response(int r) const {
    const int k = tl - ob0;
    if constexpr (L::OROWS > 1) {
      const float* J = s->rwo[r];
      if (k >= 3) return J[k] * prcp(omass());
      const V3 y = obj_inv_inertia(v3(J[0], J[1], J[2]));
      return k == 0 ? y.x : k == 1 ? y.y : y.z;
    }
    V3 wo, d;
    obj_jrow(r, &wo, &d);
    if (k >= 3) return (k == 3 ? d.x : (k == 4 ? d.y : d.z)) * prcp(omass());
    const V3 y = obj_inv_inertia(wo);
    return k == 0 ? y.x : k == 1 ? y.y : y.z;
  }

  // ---------------------------------------------------------------- test solves: Y = M~^-1 J^T, RB rows at once
  // Right-hand side q is row r0 + q: spatial force -fw on its node A and +fw on node B (contact rows) or a
  // unit joint force +-1 on node jn (limit rows).  Lane q < RB walks its own paths to the root (private
  // ut / proot slabs, so the walks run in parallel) and the root solve gives a0 per column.  The forward
  // pass is then written in joint space, y_j = (ut_j - U_j.a0 - sum_{i in anc(j)} (U_j.S_i) y_i) / D_j:
  // level by level, each lane gathers its ancestor's y values with one bpermute per column (no LDS
  // round trip or barrier per level).  y[q] = this lane's entry of Y_{r0+q} (0 off the columns).
  __device__ __forceinline__ void test_solve(int r0, int nrows_, const float* Wv, float* y) {
    MG_NC_TS
    for (int i = tl; i < L::RB * MN; i += T) s->ut(0)[i] = 0.0f;
    wsync();
    if (tl < L::RB) {
      const int r = r0 + tl;
      SV proot = szero();
      if (r < nrows_) {
        const int kind = row_kind(r);
        int nodeA = -1, nodeB = -1, jn = -1;
        float sg = 0.0f;
        SV fw = szero();
        if (kind >= 2) {
          jn = row_ref(r);
          sg = kind == 2 ? 1.0f : -1.0f;
        } else {
          const int c = r / 3;
          nodeA = cside(c, 0);
          nodeB = cside(c, 1);
          float w[6];
          row_w(r, w);
          fw = sv(v3(w[0], w[1], w[2]), v3(w[3], w[4], w[5]));
        }
        float* ut = s->ut(tl);
        // 32-lane locomotion teams (Humanoid: 35 % of the contacts are self contacts with two tree sides): both
        // sides of a contact at once.  Below their lowest common ancestor the two paths are walked in one loop
        // (two independent chains per step), and from there to the root, the map pv -> pv + U D (t - S.pv) being
        // linear, the sum of the two forces is walked once; a limit row has one path.  Same-box A/B: Humanoid
        // +1.9 %; Ant -1.3 % and ShadowHand -0.6 % (few two-sided contacts), which keep the side-by-side walks.
        if constexpr (T >= 32 && !OBJ) {
          const bool two = kind < 2 && nodeA > 0 && nodeB > 0;
          int ka = kind >= 2 ? (jn > 0 ? jn : -1) : nodeA, kb = two ? nodeB : -1;
          SV pa = kind >= 2 ? szero() : fw * -1.0f, pb = fw;
          float ta = kind >= 2 ? sg : 0.0f;
          if (kind < 2 && nodeA == 0) { proot = proot + pa; ka = -1; }
          if (kind < 2 && nodeB == 0) proot = proot + pb;
          if (kind < 2 && nodeB > 0 && !two) { ka = nodeB; pa = pb; }  // side A off the tree (ground / object)
          const unsigned long long ma = ka > 0 ? (mt->anc[ka] & ~1ull) : 0ull, mb = kb > 0 ? (mt->anc[kb] & ~1ull) : 0ull;
          const unsigned long long com = two ? (ma & mb) : 0ull;
          unsigned long long wa = ma & ~com, wb = mb & ~com;
          // below the common ancestor: both chains per step (a lane with one side left idles on the other)
          while (wa | wb) {
            const int k1 = wa ? 63 - __builtin_clzll(wa) : 0, k2 = wb ? 63 - __builtin_clzll(wb) : 0;
            const SV S1 = sv(ld3(s->S[k1]), ld3(s->S[k1] + 3)), U1 = sv(ld3(s->U[k1]), ld3(s->U[k1] + 3));
            const SV S2 = sv(ld3(s->S[k2]), ld3(s->S[k2] + 3)), U2 = sv(ld3(s->U[k2]), ld3(s->U[k2] + 3));
            const float D1 = s->Dinv[k1], D2 = s->Dinv[k2];
            if (wa) {
              const float u1 = ta - dot(S1, pa);
              atomicAdd(&ut[k1], u1);
              pa = pa + U1 * (u1 * D1);
              ta = 0.0f;
              wa &= ~(1ull << k1);
            }
            if (wb) {
              const float u2 = -dot(S2, pb);
              atomicAdd(&ut[k2], u2);
              pb = pb + U2 * (u2 * D2);
              wb &= ~(1ull << k2);
            }
          }
          SV pv = two ? pa + pb : pa;
          for (unsigned long long wc = com; wc;) {
            const int k = 63 - __builtin_clzll(wc);
            wc &= ~(1ull << k);
            const SV Sk = sv(ld3(s->S[k]), ld3(s->S[k] + 3)), Uk = sv(ld3(s->U[k]), ld3(s->U[k] + 3));
            const float uk = -dot(Sk, pv);
            atomicAdd(&ut[k], uk);
            pv = pv + Uk * (uk * s->Dinv[k]);
          }
          if (ka > 0 || two) proot = proot + pv;
        } else {
        for (int side = 0; side < 3; side++) {
          int k0;
          SV pv;
          float tq = 0.0f;
          if (side == 0) { k0 = nodeA; pv = fw * -1.0f; }
          else if (side == 1) { k0 = nodeB; pv = fw; }
          else { k0 = jn; pv = szero(); tq = sg; }
          if (k0 < 0 || (side == 2 && k0 == 0)) continue;
          if (k0 == 0) {  // force on the root body: straight into the root's bias
            proot = proot + pv;
            continue;
          }
          // the path to the root is the ancestor mask (parents precede children, checked at sim
          // creation), so the next node's S / U / D^-1 are loaded while this one is processed; the
          // ut accumulations are fire-and-forget LDS adds (program order per lane, as the oracle)
          unsigned long long path = mt->anc[k0] & ~1ull;
          int k = 63 - __builtin_clzll(path);
          SV Sk = sv(ld3(s->S[k]), ld3(s->S[k] + 3)), Uk = sv(ld3(s->U[k]), ld3(s->U[k] + 3));
          float Dk = s->Dinv[k];
          while (true) {
            path &= ~(1ull << k);
            const int kn = path ? 63 - __builtin_clzll(path) : 0;
            // the next node's terms loaded unconditionally (node 0's rows when the path ends: valid, unused; same-box
            // A/B against a guarded load: ShadowHand +1.6 %, Ant +0.2 %)
            const SV Sn = sv(ld3(s->S[kn]), ld3(s->S[kn] + 3)), Un = sv(ld3(s->U[kn]), ld3(s->U[kn] + 3));
            const float Dn = s->Dinv[kn];
            const float uk = tq - dot(Sk, pv);
            atomicAdd(&ut[k], uk);
            pv = pv + Uk * (uk * Dk);
            tq = 0.0f;
            if (kn == 0) break;
            k = kn; Sk = Sn; Uk = Un; Dk = Dn;
          }
          proot = proot + pv;
        }
        }
      }
      float* pr = s->tsroot(tl);
      pr[0] = proot.a.x; pr[1] = proot.a.y; pr[2] = proot.a.z;
      pr[3] = proot.l.x; pr[4] = proot.l.y; pr[5] = proot.l.z;
    }
    wsync();
    ph_mark(10);
    // base_q = ut_j - U_j.a0 (joint lanes) or a0[tl] (root lanes), both as ut + Wv.p0 (see aba())
    // rem_q starts at base_q and loses C_ji y_i as the ancestors' values arrive
    float rem[L::RB], yv[L::RB];
#pragma unroll
    for (int q = 0; q < L::RB; q++) {
      const float* p0 = s->tsroot(q);
      float b = node > 0 ? s->ut(q)[node] : 0.0f;
      b += Wv[0] * p0[0] + Wv[1] * p0[1] + Wv[2] * p0[2] + Wv[3] * p0[3] + Wv[4] * p0[4] + Wv[5] * p0[5];
      rem[q] = b;
      yv[q] = 0.0f;
    }
    ph_mark(11);
    // proper ancestors below the root, visited in increasing depth (= increasing index)
    unsigned long long path = node > 0 ? (mt->anc[node] & ~1ull & ~(1ull << node)) : 0ull;
    // the level's y values are published in the (now read) ut slab, RB floats per node, and every deeper
    // lane reads its ancestor's row: a few wide LDS accesses per level instead of RB bpermutes
    float* ybuf = s->ut(0);
    static_assert(L::kUtFloats >= L::RB * MN, "y rows must fit the ut slab");
    wsync();
    for (int lev = 1; lev <= maxdepth; lev++) {
      if (node > 0 && depth == lev) {
#pragma unroll
        for (int q = 0; q < L::RB; q++) {
          yv[q] = rem[q] * Dinv;
          ybuf[L::RB * node + q] = yv[q];
        }
      }
      wsync();
      if (lev < maxdepth && node > 0 && depth > lev) {
        const int an = __builtin_ctzll(path);
        path &= path - 1;
        const float C = dot(U, sv(ld3(s->S[an]), ld3(s->S[an] + 3)));
        const float* ya = ybuf + L::RB * an;
#pragma unroll
        for (int q = 0; q < L::RB; q++) rem[q] -= C * ya[q];
      }
    }
    ph_mark(12);
#pragma unroll
    for (int q = 0; q < L::RB; q++) {
      float v = (freeb && tl < 6) ? rem[q] : yv[q];
      y[q] = tl < nv ? v : 0.0f;
    }
  }

  // side k of contact c: 0 node A, 1 node B, 2 geom A, 3 geom B
  __device__ __forceinline__ int cside(int c, int k) const { return (int)(int8_t)(s->cside[c] >> (8 * k)); }
  // row r -> kind (0 normal, 1 friction, 2 lower limit, 3 upper limit) and ref (contact / node).
  // Rows are [n, t1, t2] per contact, then the joint limits (oracle order).
  __device__ __forceinline__ int row_kind(int r) const { return r < 3 * ncr ? (r % 3 == 0 ? 0 : 1) : (s->lm(r - 3 * ncr) & 3); }
  __device__ __forceinline__ int row_ref(int r) const { return r < 3 * ncr ? r / 3 : (s->lm(r - 3 * ncr) >> 4); }
  // spatial direction of contact row r at the team origin: w = [(p - o) x d; d]
  __device__ __forceinline__ void row_w(int r, float* w) const {
    const int c = r / 3, k = r - 3 * c;
    V3 t1, t2;
    s->tangents(c, &t1, &t2);
    const V3 d = k == 0 ? ld3(s->cn[c]) : (k == 1 ? t1 : t2), q = ld3(s->cp[c]) - org, mo = cross(q, d);
    w[0] = mo.x; w[1] = mo.y; w[2] = mo.z; w[3] = d.x; w[4] = d.y; w[5] = d.z;
  }
  // Jacobian code of this lane for row r: 0 none, 1 +, 2 - (contact rows: +-Sl.w; limit rows: +-1
  // on the DOF's lane)
  __device__ __forceinline__ int jac_code(int r) const {
    if (tl >= nv || (OBJ && objl)) return 0;
    const int kind = row_kind(r);
    if (kind >= 2) return (node > 0 && node == row_ref(r)) ? (kind == 2 ? 1 : 2) : 0;
    const int c = r / 3, A = cside(c, 0), B = cside(c, 1);
    float sgn;
    if (freeb && tl < 6) sgn = (A >= 0 ? 1.0f : 0.0f) - (B >= 0 ? 1.0f : 0.0f);
    else if (node <= 0) return 0;
    else sgn = (in_path(A, node) ? 1.0f : 0.0f) - (in_path(B, node) ? 1.0f : 0.0f);
    return sgn > 0.0f ? 1 : (sgn < 0.0f ? 2 : 0);
  }
  // J_r[tl] from the lane's code (object lanes: the stored object part)
  __device__ __forceinline__ float jac_value(int r, int code) const {
    if (OBJ && objl) {
      if constexpr (L::OROWS > 1) return r >= 3 * ncr ? 0.0f : s->rwo[r][tl - ob0];
      if (r >= 3 * ncr) return 0.0f;
      V3 wo, d;
      obj_jrow(r, &wo, &d);
      const int k = tl - ob0;
      return k == 0 ? wo.x : k == 1 ? wo.y : k == 2 ? wo.z : k == 3 ? d.x : k == 4 ? d.y : d.z;
    }
    if (code == 0) return 0.0f;
    if (r >= 3 * ncr) return code == 1 ? 1.0f : -1.0f;
    float w[6];
    row_w(r, w);
    const float d = Sl[0] * w[0] + Sl[1] * w[1] + Sl[2] * w[2] + Sl[3] * w[3] + Sl[4] * w[4] + Sl[5] * w[5];
    return code == 1 ? d : -d;
  }

  // J_r[lane] for the 3 rows r0 .. r0 + 2 of a test-solve batch (r0 a multiple of 3).  Contact rows come in aligned
  // triples (n, t1, t2 of contact r0 / 3): they share the lane's sign and the point-velocity vector
  // g = Sl_ang x (p - o) + Sl_lin, so J_r = sign (d_r . g) (= sign Sl . [(p - o) x d_r; d_r]).
  // Limit rows: +-1 on the DOF's lane.  Object lanes: the stored object part of the contact rows.
  __device__ __forceinline__ void batch_jacobians(int r0, int nrows_, float* J) const {
    MG_NC_JAC
#pragma unroll
    for (int q = 0; q < 3; q++) J[q] = 0.0f;
    if (OBJ && objl) {
      if constexpr (L::OROWS > 1) {
        if (r0 < 3 * ncr)
          for (int q = 0; q < 3; q++) J[q] = s->rwo[r0 + q][tl - ob0];
        return;
      }
      if (r0 < 3 * ncr) {
        const int k = tl - ob0;
        for (int q = 0; q < 3; q++) {
          V3 wo, d;
          obj_jrow(r0 + q, &wo, &d);
          J[q] = k == 0 ? wo.x : k == 1 ? wo.y : k == 2 ? wo.z : k == 3 ? d.x : k == 4 ? d.y : d.z;
        }
      }
      return;
    }
    if (tl >= nv) return;
    if (r0 < 3 * ncr) {
      const int c = r0 / 3, A = cside(c, 0), B = cside(c, 1);
      float sgn;
      if (freeb && tl < 6) sgn = (A >= 0 ? 1.0f : 0.0f) - (B >= 0 ? 1.0f : 0.0f);
      else if (node <= 0) return;
      else sgn = (in_path(A, node) ? 1.0f : 0.0f) - (in_path(B, node) ? 1.0f : 0.0f);
      if (sgn == 0.0f) return;
      const V3 g = cross(v3(Sl[0], Sl[1], Sl[2]), ld3(s->cp[c]) - org) + v3(Sl[3], Sl[4], Sl[5]);
      J[0] = sgn * dot(ld3(s->cn[c]), g);
      V3 t1, t2;
      s->tangents(c, &t1, &t2);
      J[1] = sgn * dot(t1, g);
      J[2] = sgn * dot(t2, g);
    } else {
#pragma unroll
      for (int q = 0; q < 3; q++) {
        const int r = r0 + q;
        if (r < nrows_ && node > 0) {
          const int meta = s->lm(r - 3 * ncr);
          if ((meta >> 4) == node) J[q] = (meta & 3) == 2 ? 1.0f : -1.0f;
        }
      }
    }
  }

  // ---------------------------------------------------------------- collision -> LDS contact list
  __device__ __forceinline__ void geom_world(int g, V3* cw, M3* Rg) const {
    const int nd = mt->gnode[g];
    const float* gf = mt->gf[g];
    M3 Rn, Rl;
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) {
        Rn.m[a][b] = s->R[nd][3 * a + b];
        Rl.m[a][b] = gf[3 + 3 * a + b];
      }
    *cw = ld3(s->x[nd]) + mul(Rn, ld3(gf));
    *Rg = mul(Rn, Rl);
  }
  // world frames of the geoms, staged once per substep by collide() (lane per geom) in the team's
  // union storage (dead between the ABA and build_rows); rows of 13 floats (odd stride): centre, R
  static constexpr int GW = 13;
  __device__ __forceinline__ float* gw_tile() const { return s->gw(); }
  __device__ __forceinline__ void geom_staged(int g, V3* c, M3* Rg) const {
    const float* w = gw_tile() + GW * g;
    *c = v3(w[0], w[1], w[2]);
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) Rg->m[a][b] = w[3 + 3 * a + b];
  }
  __device__ __forceinline__ bool geom_segment(int g, V3* a, V3* b, float* r) const {
    V3 c;
    M3 Rg;
    geom_staged(g, &c, &Rg);
    int ty = mt->gtype[g];
    const float* gs = mt->gf[g] + 12;
    if (ty == MG_GT_SPHERE) { *a = c; *b = c; *r = gs[0]; return true; }
    if (ty == MG_GT_CAPSULE) {
      V3 ax = v3(Rg.m[0][2], Rg.m[1][2], Rg.m[2][2]) * gs[1];
      *a = c - ax; *b = c + ax; *r = gs[0];
      return true;
    }
    return false;
  }

  // candidate q of articulation geom g against the object box (oracle geom_object): sphere/capsule
  // -> one closest-point candidate; box -> its 8 vertices vs the object, then the object's 8 vertices
  // vs the geom (normal flipped).  Normal points from the object (B) to the geom (A).
  __device__ __forceinline__ bool obj_candidate(int g, int q, V3 c, const M3& Rg, V3* pt, V3* nrm, float* dist) const {
    const V3 hb = osize();
    const int ty = mt->gtype[g];
    const float* gs = mt->gf[g] + 12;
    const bool round = ty == MG_GT_SPHERE || ty == MG_GT_CAPSULE;
    const V3 hg = v3(gs[0], gs[1], gs[2]);
    if (!round && q == 16) {  // edge against edge, in the object frame
      M3 Rt;
      for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) Rt.m[a][b] = oR.m[b][a];
      V3 pe, ne;
      float de;
      if (!box_box_edge(mulT(oR, c - op), mul(Rt, Rg), hg, hb, p->contact_offset, &pe, &ne, &de)) return false;
      *pt = mul(oR, pe) + op;
      *nrm = mul(oR, ne);
      *dist = de;
      return true;
    }
    // every other candidate is one point against one box: the segment's closest point (sphere / capsule) or a
    // geom vertex against the object box, an object vertex against the geom box.  The three set up the query
    // (point P in the box's frame, the box, the frame's rotation / origin, radius, normal sign) and share one
    // point_box and the output transform, so a pass whose lanes mix them runs point_box once, not three times.
    V3 P, hx, cf;
    M3 Rf;
    float r = 0.0f, sgn = 1.0f;
    const int v = q & 7;
    if (round) {
      const float hl = ty == MG_GT_CAPSULE ? gs[1] : 0.0f;
      const V3 ax = v3(Rg.m[0][2], Rg.m[1][2], Rg.m[2][2]) * hl;
      const V3 al = mulT(oR, (c - ax) - op), bl = mulT(oR, (c + ax) - op), u = bl - al;
      r = gs[0];
      bool inside;
      float t = seg_box_t(al, u, hb, &inside);
      if (inside) {  // the core inside the cube: the seg_box_sat face (its own point, normal and depth)
        const int f = seg_box_sat(al, u, hb, &t);
        P = al + u * t;
        V3 nb, cb;
        *dist = box_face_point(P, hb, f, &nb, &cb) - r;
        *pt = mul(oR, ((P - nb * r) + cb) * 0.5f) + op;
        *nrm = mul(oR, nb);
        return true;
      }
      P = al + u * t;
    } else if (q < 8) {
      const V3 l = v3((v & 1 ? 1.f : -1.f) * hg.x, (v & 2 ? 1.f : -1.f) * hg.y, (v & 4 ? 1.f : -1.f) * hg.z);
      P = mulT(oR, (c + mul(Rg, l)) - op);
    } else {
      const V3 l = v3((v & 1 ? 1.f : -1.f) * hb.x, (v & 2 ? 1.f : -1.f) * hb.y, (v & 4 ? 1.f : -1.f) * hb.z);
      P = mulT(Rg, (mul(oR, l) + op) - c);
      sgn = -1.0f;
    }
    const bool geom_box = !round && q >= 8;
    hx = geom_box ? hg : hb;
    cf = geom_box ? c : op;
#pragma unroll
    for (int a = 0; a < 3; a++)
#pragma unroll
      for (int b = 0; b < 3; b++) Rf.m[a][b] = geom_box ? Rg.m[a][b] : oR.m[a][b];
    V3 nb, cb;
    *dist = point_box(P, hx, &nb, &cb) - r;
    *pt = mul(Rf, ((P - nb * r) + cb) * 0.5f) + cf;
    *nrm = mul(Rf, nb) * sgn;
    return true;
  }

  // The convex-mesh geom against the object (oracle geom_object / geom_object_convex, MG_GT_CONVEX branches):
  //   block: the hull's vertices against the box, then the box's 8 vertices against the hull's faces;
  //   pen:   the hull's vertices against its segment, then its two end spheres against the faces;
  //   egg:   the faces against the ellipsoid's support points.
  // Normal from the object to the geom.  Hull vertex q against the object (block / pen), lane per vertex:
  __device__ __forceinline__ bool hull_vertex_candidate(int q, V3 c, const M3& Rg, V3* pt, V3* nrm, float* dist) const {
    const V3 w = c + mul(Rg, ld3(mt->hv[q]));  // the tile's copy of m->hull_vert (LDS)
    if constexpr (OBJ == MG_GT_BOX) {
      const V3 pl = mulT(oR, w - op);
      V3 nb, cb;
      *dist = point_box(pl, osize(), &nb, &cb);
      *pt = mul(oR, (pl + cb) * 0.5f) + op;
      *nrm = mul(oR, nb);
      return true;
    } else {
      const V3 os = osize();
      const float ro = os.x;
      const V3 oz = v3(oR.m[0][2], oR.m[1][2], oR.m[2][2]) * os.y;
      const V3 p0 = op - oz, p1 = op + oz;
      float ss, tt;
      closest_seg_seg_t(w, w, p0, p1, &ss, &tt);
      const V3 qq = p0 + (p1 - p0) * tt, dv = w - qq;
      const float dl = sqrtf(dot(dv, dv));
      if (!(dl > 1e-9f)) return false;
      *nrm = dv * prcp(dl);
      *pt = (w + (qq + *nrm * ro)) * 0.5f;
      *dist = dl - ro;
      return true;
    }
  }
  // object point k (block: box vertex k; pen: end k; egg: unused) in the geom frame
  __device__ __forceinline__ V3 hull_object_point(int k, V3 c, const M3& Rg) const {
    const V3 os = osize();
    if constexpr (OBJ == MG_GT_BOX) {
      const V3 l = v3((k & 1 ? 1.f : -1.f) * os.x, (k & 2 ? 1.f : -1.f) * os.y, (k & 4 ? 1.f : -1.f) * os.z);
      return mulT(Rg, (mul(oR, l) + op) - c);
    } else {
      const V3 oz = v3(oR.m[0][2], oR.m[1][2], oR.m[2][2]) * os.y;
      return mulT(Rg, (k == 0 ? op - oz : op + oz) - c);
    }
  }
  // egg: its support point (geom frame) farthest along -n (n a geom-frame face normal); cl / Rl: the egg's
  // centre and axes in the geom frame
  __device__ __forceinline__ V3 egg_support_geom(V3 n, V3 cl, const M3& Rl) const {
    const V3 os = osize();
    const V3 ne = mulT(Rl, n * -1.0f);
    const V3 qe = v3(os.x * os.x * ne.x, os.y * os.y * ne.y, os.z * os.z * ne.z);
    const float nn = sqrtf(qe.x * ne.x + qe.y * ne.y + qe.z * ne.z);
    const V3 se = nn < 1e-30f ? v3(0, 0, 0) : qe * (1.0f / nn);
    return mul(Rl, se) + cl;
  }

  // object-contact candidates of an articulation geom of type ty (oracle obj_candidates): block
  // sphere/capsule 1, box 17 (vertex tests both ways, edge-edge); pen sphere/capsule 1 (segment-segment),
  // box 3 (closest point + the two ends); egg 1 (GJK / MPR); the convex-mesh geom as counted below
  __device__ __forceinline__ int ocand_count(int ty) const {
    const bool round = ty == MG_GT_SPHERE || ty == MG_GT_CAPSULE;
    constexpr int ot = OBJ;
    if (ty == MG_GT_CONVEX)  // block: hull vertices + the box's 8 + exact; pen: hull vertices + its 2 ends + exact
      return ot == MG_GT_BOX ? mt->hnv + 9 : (ot == MG_GT_CAPSULE ? mt->hnv + 3 : 1);
    if (!round && ty != MG_GT_BOX) return 0;
    if (ot == MG_GT_BOX) return round ? 1 : 17;  // box: 8 + 8 vertex-face, 1 edge-edge
    if (ot == MG_GT_CAPSULE) return round ? 1 : 3;
    return 1;
  }
  // bounding radius of the object (broadphase cull)
  __device__ __forceinline__ float obj_radius() const {
    const V3 e = osize();
    constexpr int ot = OBJ;
    if (ot == MG_GT_BOX) return sqrtf(dot(e, e));
    if (ot == MG_GT_CAPSULE) return e.x + e.y;
    return fmaxf(e.x, fmaxf(e.y, e.z));
  }
  // candidate q of geom g against the pen / egg (oracle geom_object_convex); false = no candidate
  __device__ __forceinline__ bool obj_candidate_convex(int g, int q, V3 c, const M3& Rg, V3* pt, V3* nrm, float* dist) const {
    const V3 os = osize();
    const int ty = mt->gtype[g];
    const float* gs = mt->gf[g] + 12;
    const bool round = ty == MG_GT_SPHERE || ty == MG_GT_CAPSULE;
    if constexpr (OBJ == MG_GT_ELLIPSOID) {
      // the core as five 3-vectors in the object frame (convex.hpp cvx_contact_v, inlined)
      int kind;
      V3 a0, a1, a2 = v3(0, 0, 0), a3 = v3(0, 0, 0), a4 = v3(0, 0, 0);
      float r = 0.0f;
      if (round) {
        const float hl = ty == MG_GT_CAPSULE ? gs[1] : 0.0f;
        const V3 ax = v3(Rg.m[0][2], Rg.m[1][2], Rg.m[2][2]) * hl;
        kind = 0;
        a0 = mulT(oR, (c - ax) - op);
        a1 = mulT(oR, (c + ax) - op);
        r = gs[0];
      } else {
        kind = 1;
        a0 = mulT(oR, c - op);
        M3 Rt;
        for (int a = 0; a < 3; a++)
          for (int b = 0; b < 3; b++) Rt.m[a][b] = oR.m[b][a];
        const M3 Rl = mul(Rt, Rg);  // box axes in the object frame (columns)
        a1 = v3(gs[0], gs[1], gs[2]);
        a2 = v3(Rl.m[0][0], Rl.m[1][0], Rl.m[2][0]);
        a3 = v3(Rl.m[0][1], Rl.m[1][1], Rl.m[2][1]);
        a4 = v3(Rl.m[0][2], Rl.m[1][2], Rl.m[2][2]);
      }
      const CvxHit hit = cvx_contact_v(kind, a0, a1, a2, a3, a4, r, os, p->contact_offset);
      *dist = hit.d;
      *pt = mul(oR, hit.pt) + op;
      *nrm = mul(oR, hit.nrm);
      return true;
    }
    // pen: capsule of radius os.x along the object's z, half length os.y
    const float ro = os.x;
    const V3 oz = v3(oR.m[0][2], oR.m[1][2], oR.m[2][2]) * os.y;
    const V3 p0 = op - oz, p1 = op + oz;
    if (round) {
      const float hl = ty == MG_GT_CAPSULE ? gs[1] : 0.0f, r = gs[0];
      const V3 ax = v3(Rg.m[0][2], Rg.m[1][2], Rg.m[2][2]) * hl;
      const V3 a0 = c - ax, a1 = c + ax;
      float ss, tt;
      closest_seg_seg_t(a0, a1, p0, p1, &ss, &tt);
      const V3 pa = a0 + (a1 - a0) * ss, pb = p0 + (p1 - p0) * tt, dv = pa - pb;
      const float dl = sqrtf(dot(dv, dv));
      if (!(dl > 1e-9f)) return false;
      *nrm = dv * prcp(dl);
      *pt = ((pa - *nrm * r) + (pb + *nrm * ro)) * 0.5f;
      *dist = dl - r - ro;
      return true;
    }
    const V3 hg = v3(gs[0], gs[1], gs[2]);
    const V3 P0 = mulT(Rg, p0 - c), u = mulT(Rg, p1 - p0);
    bool inside;
    float ts = seg_box_t(P0, u, hg, &inside);
    // the core inside the box: every candidate against the seg_box_sat face (q = 0 its deepest end, the other
    // end by its own depth behind that face)
    const int face = inside ? seg_box_sat(P0, u, hg, &ts) : -1;
    if ((q == 1 && ts < 0.01f) || (q == 2 && ts > 0.99f)) return false;
    const float t = q == 0 ? ts : (q == 1 ? 0.0f : 1.0f);
    const V3 P = P0 + u * t;
    V3 nb, cb;
    *dist = (inside ? box_face_point(P, hg, face, &nb, &cb) : point_box(P, hg, &nb, &cb)) - ro;
    *pt = mul(Rg, ((P - nb * ro) + cb) * 0.5f) + c;
    *nrm = mul(Rg, nb) * -1.0f;
    return true;
  }

  // The exact hull candidates of this substep (hull.hpp), before the tree phases: the convex-mesh geom is on the
  // hand's fixed root (checked at launch), so its world frame (built as fk() + geom_world() build it) and the
  // object's pose are the ones collide() sees, and the narrowphase runs where little else is live.  The
  // broadphase is collide()'s (the geom's bounding sphere, then its box against the object's sphere).
  __device__ __forceinline__ void hull_stage() {
    if constexpr (L::HX > 0) {
      const int g = mt->hullg;
      int nx = 0;
      bool near = false;  // the object within the offset of the hull's planes (else collide() skips the hull)
      float res[14];
      V3 c = v3(0, 0, 0);
      M3 Rg;
#ifdef MG_PHASE_TIMING
      // profiling build: the narrowphase's GJK / MPR / rest (hull_core_contacts) and the plane bound, per team
      unsigned hcyc[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
      const unsigned long long th0 = __builtin_amdgcn_s_memtime();
#endif
      if (g >= 0 && (mt->gfil[g] & MG_COLLIDE_OBJECT)) {
        const M3 R0 = quat_to_mat(q0[0], q0[1], q0[2], q0[3]);
        const float* gf = mt->gf[g];
        M3 Rl;
        for (int a = 0; a < 3; a++)
          for (int b = 0; b < 3; b++) Rl.m[a][b] = gf[3 + 3 * a + b];
        c = p0 + mul(R0, ld3(gf));
        Rg = mul(R0, Rl);
        const float ro = obj_radius(), off = p->contact_offset;
        const V3 dc = c - op;
        const float reach = gf[15] + ro + off;
        if (dot(dc, dc) <= reach * reach && hull_box_near(c, Rg, ld3(gf + 12), op, ro, off)) {
          const M3 oRs = quat_to_mat(oq[0], oq[1], oq[2], oq[3]);
          HullCore B;
          float rB;
          const V3 os = osize();
          if constexpr (OBJ == MG_GT_BOX) {
            B.kind = 1;
            B.c = mulT(Rg, op - c);
            for (int a = 0; a < 3; a++)
              for (int b = 0; b < 3; b++)
                B.R.m[a][b] = Rg.m[0][a] * oRs.m[0][b] + Rg.m[1][a] * oRs.m[1][b] + Rg.m[2][a] * oRs.m[2][b];
            const float mg = fminf(HULL_MARGIN, 0.5f * fminf(os.x, fminf(os.y, os.z)));
            B.h = v3(os.x - mg, os.y - mg, os.z - mg);
            rB = mg;
          } else {
            const V3 oz = v3(oRs.m[0][2], oRs.m[1][2], oRs.m[2][2]) * os.y;
            B.kind = 0;
            B.p0 = mulT(Rg, (op - oz) - c);
            B.p1 = mulT(Rg, (op + oz) - c);
            rB = os.x;
          }
          // a lower bound of the object's distance to the hull from its plane distances (each plane's distance is
          // at most the true one): the cube's centre minus its circumradius, or the pen's segment by max over the
          // planes of the nearer end (max_f min_t <= min_t max_f); at or beyond the offset there is no contact
          float lb = -3.0e38f;
          const int np = m->hull_num_planes;
#pragma unroll 4
          for (int k = 0; k < (MG_MAX_HULL_PLANES + T - 1) / T; k++) {  // batches of loads, then the reduction
            const int f = tl + k * T;
            if (f < np) {
              const float4 q = *reinterpret_cast<const float4*>(m->hull_plane[f]);
              const V3 nf = v3(q.x, q.y, q.z);
              const float sd = B.kind == 1 ? dot(nf, B.c) - q.w : fminf(dot(nf, B.p0), dot(nf, B.p1)) - q.w;
              lb = fmaxf(lb, sd);
            }
          }
          lb = team_max_dpp<T>(lb);
          lb -= B.kind == 1 ? sqrtf(dot(os, os)) : rB;
          // the bound is fp32 on another path than the candidates' own distances (and the oracle has no such
          // cull): a 1 um guard band keeps a candidate just under the offset from being dropped by rounding
          if (lb < off + 1e-6f) {
#ifdef MG_PHASE_TIMING
            hcyc[3] += (unsigned)(__builtin_amdgcn_s_memtime() - th0);
            nx = hull_core_contacts<T>(mt->hv, mt->hnv, ld3(mt->hctr), m->hull_plane, np, tl, tb, B, rB, off, res, hcyc);
#else
            nx = hull_core_contacts<T>(mt->hv, mt->hnv, ld3(mt->hctr), m->hull_plane, np, tl, tb, B, rB, off, res);
#endif
            near = true;
          }
        }
      }
#ifdef MG_PHASE_TIMING
      for (int k = 0; k < 8; k++) {  // the wave's slowest team (every lane holds its team's value; 0 if not near)
        unsigned wmax = 0;
        for (int q = 0; q < 64; q += T) {
          const unsigned cq = (unsigned)__builtin_amdgcn_readlane((int)hcyc[k], q);
          wmax = cq > wmax ? cq : wmax;
        }
        ph[23 + k] = __builtin_amdgcn_readfirstlane(ph[23 + k] + wmax);
      }
#endif
      if (tl == 0) {
        for (int i = 0; i < nx; i++) {
          const V3 pw = mul(Rg, ld3(res + 7 * i)) + c, nw = mul(Rg, ld3(res + 7 * i + 3));
          s->hx[i][0] = pw.x; s->hx[i][1] = pw.y; s->hx[i][2] = pw.z;
          s->hx[i][3] = nw.x; s->hx[i][4] = nw.y; s->hx[i][5] = nw.z;
          s->hx[i][6] = res[7 * i + 6];
        }
        s->hxn = near ? nx : -1;
      }
    }
  }

  // The egg's narrowphase, staged right after fk() (fp32, convex.hpp): its candidates are the geoms that pass
  // collide()'s broadphase (bounding sphere against the egg's; sphere / capsule / box geoms, one candidate each,
  // geom order), evaluated where only the joint state is live -- fk()'s register outputs are reloaded from their
  // LDS copies afterwards (reload_tree) -- so the narrowphase's working set does not spill the tree state the
  // ABA and the rows need.  The results wait in storage that is dead until build_rows(): point -> ct1[f],
  // normal -> ct2[f], gap -> lmeta[f] (bits), geom -> lmeta[MN - 1 + f], count -> nrows; collide() emits them
  // in its object pass, in the same order as the unstaged candidates.
  __device__ __forceinline__ void egg_stage() {
    if constexpr (OBJ == MG_GT_ELLIPSOID) {
      static_assert(MG <= MC && MG <= MN - 1 && MG <= T, "the egg's staged candidates must fit one team pass");
      const float ro = obj_radius(), off = p->contact_offset;
      const int G = mt->ng;
      bool ok = false;
      if (tl < G) {
        const int gt = mt->gtype[tl];
        if ((mt->gfil[tl] & MG_COLLIDE_OBJECT) && (gt == MG_GT_SPHERE || gt == MG_GT_CAPSULE || gt == MG_GT_BOX)) {
          V3 c;
          M3 Rg;
          geom_world(tl, &c, &Rg);
          const V3 dc = c - op;
          const float reach = mt->gf[tl][15] + ro + off;
          ok = dot(dc, dc) <= reach * reach;
        }
      }
      constexpr unsigned long long tmask = T >= 64 ? ~0ull : ((1ull << T) - 1ull);
      const unsigned long long live = (__ballot(ok) >> tb) & tmask;
      const int NC = __popcll(live);
      if (tl < NC) {
        unsigned long long mm = live;
        for (int k = 0; k < tl; k++) mm &= mm - 1;
        const int g = __builtin_ctzll(mm);
        V3 c, pt, nrm;
        M3 Rg;
        float d;
        geom_world(g, &c, &Rg);
        obj_candidate_convex(g, 0, c, Rg, &pt, &nrm, &d);
        s->ct1[tl][0] = pt.x; s->ct1[tl][1] = pt.y; s->ct1[tl][2] = pt.z;
        s->ct2[tl][0] = nrm.x; s->ct2[tl][1] = nrm.y; s->ct2[tl][2] = nrm.z;
        s->lmeta[tl] = __float_as_int(d);
        s->lmeta[MN - 1 + tl] = g;
      }
      if (tl == 0) s->nrows = NC;
    }
  }
  // fk()'s register outputs (R, x, V; S on joint lanes) again, from the copies it stored in the LDS
  __device__ __forceinline__ void reload_tree() {
    asm volatile("" ::: "memory");
    R = M3{};
    x = v3(0, 0, 0);
    V = S = szero();
    if (node >= 0) {
      for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) R.m[a][b] = s->R[node][3 * a + b];
      x = ld3(s->x[node]);
      V = sv(ld3(s->V[node]), ld3(s->V[node] + 3));
    }
    if (node > 0) S = sv(ld3(s->S[node]), ld3(s->S[node] + 3));
  }

  __device__ __forceinline__ void put_contact(int slot, V3 pt, V3 n, float d, int A, int gA, int B, int gB) {
    s->cp[slot][0] = pt.x; s->cp[slot][1] = pt.y; s->cp[slot][2] = pt.z;
    s->cn[slot][0] = n.x; s->cn[slot][1] = n.y; s->cn[slot][2] = n.z;
    s->set_gap(slot, d);
    s->cside[slot] = (A & 0xff) | ((B & 0xff) << 8) | ((gA & 0xff) << 16) | ((gB & 0xff) << 24);
  }

  __device__ __forceinline__ void collide() {
    const int cap = p->max_contacts < MC ? p->max_contacts : MC;
    const float off = p->contact_offset;
    int base = 0;
    const int G = mt->ng;
    static_assert(L::kGwFloats >= MG * GW, "geom frames must fit the team's union storage");
    if constexpr (L::kCompact && L::kGwInA) {
      // the frames go to region A over the poses they are built from: every lane reads its geoms' poses first
      constexpr int GPL = (MG + T - 1) / T;
      V3 cs[GPL];
      M3 Rs[GPL];
#pragma unroll
      for (int j = 0; j < GPL; j++) {
        cs[j] = v3(0, 0, 0);
        if (tl + j * T < G) geom_world(tl + j * T, &cs[j], &Rs[j]);
      }
      wsync();
#pragma unroll
      for (int j = 0; j < GPL; j++) {
        const int g = tl + j * T;
        if (g < G) {
          float* w = gw_tile() + GW * g;
          w[0] = cs[j].x; w[1] = cs[j].y; w[2] = cs[j].z;
          for (int a = 0; a < 3; a++)
            for (int b = 0; b < 3; b++) w[3 + 3 * a + b] = Rs[j].m[a][b];
        }
      }
    } else {
      for (int g = tl; g < G; g += T) {
        V3 c;
        M3 Rg;
        geom_world(g, &c, &Rg);
        float* w = gw_tile() + GW * g;
        w[0] = c.x; w[1] = c.y; w[2] = c.z;
        for (int a = 0; a < 3; a++)
          for (int b = 0; b < 3; b++) w[3 + 3 * a + b] = Rg.m[a][b];
      }
    }
    wsync();
    ph_mark(31);  // (profiling build: the geom frames' staging, apart from the ground candidates)
    // ground contacts: lane per geom, up to 8 candidates each, emitted in geom order.
    // pass 1 counts, a team scan places them, pass 2 recomputes and writes (no private arrays).
    // spheres and capsules only (the locomotion models): at most two candidates per geom, kept in registers,
    // one pass (same-box A/B against the two passes: Ant +2.3 %, Ant 16,384 +1.9 %, MA-Ant +2.4 %, Humanoid +1.2 %)
    if (mt->ground_round) {
      for (int g0 = 0; g0 < G; g0 += T) {
        const int g = g0 + tl;
        V3 e0 = v3(0, 0, 0), e1 = v3(0, 0, 0);
        float r = 0.0f, d0 = 1e30f, d1 = 1e30f;
        if (g < G && (mt->gfil[g] & MG_COLLIDE_GROUND)) {
          V3 c;
          M3 Rg;
          geom_staged(g, &c, &Rg);
          if (c.z - mt->gf[g][15] < off) {
            const float* gs = mt->gf[g] + 12;
            r = gs[0];
            if (mt->gtype[g] == MG_GT_CAPSULE) {
              const V3 ax = v3(Rg.m[0][2], Rg.m[1][2], Rg.m[2][2]) * gs[1];
              e0 = c - ax;
              e1 = c + ax;
              d1 = e1.z - r;
            } else {
              e0 = c;
            }
            d0 = e0.z - r;
          }
        }
        const bool k0 = d0 < off, k1 = d1 < off;
        const int cnt = (k0 ? 1 : 0) + (k1 ? 1 : 0);
        int scan_tot;
        const int incl = team_scan_bits<T, 2>(cnt, scan_tot);
        const int slot0 = base + incl - cnt;
        base += scan_tot;
        if (k0 && slot0 < cap) put_contact(slot0, v3(e0.x, e0.y, e0.z - r), v3(0, 0, 1), d0, mt->gnode[g], g, -1, -1);
        const int s1 = slot0 + (k0 ? 1 : 0);
        if (k1 && s1 < cap) put_contact(s1, v3(e1.x, e1.y, e1.z - r), v3(0, 0, 1), d1, mt->gnode[g], g, -1, -1);
      }
    } else
    for (int g0 = 0; g0 < G; g0 += T) {
      const int g = g0 + tl;
      V3 c = v3(0, 0, 0);
      M3 Rg;
      int ty = -1;
      if (g < G && (mt->gfil[g] & MG_COLLIDE_GROUND)) {
        geom_staged(g, &c, &Rg);
        // every candidate's gap is >= c.z - bounding radius: geoms that high cannot touch the plane; a box's lowest
        // corner exactly (Cartpole's 8 m rail: its bounding radius reaches the plane from any height), the same test
        // its corner loop would fail, so the same contacts
        if (c.z - mt->gf[g][15] < off) ty = mt->gtype[g];
        if (OBJ == 0 && ty == MG_GT_BOX) {  // (the hand instances' box geoms pass the radius test rarely: left as is)
          const float* hb = mt->gf[g] + 12;
          const float zlow = c.z - (fabsf(Rg.m[2][0]) * hb[0] + fabsf(Rg.m[2][1]) * hb[1] + fabsf(Rg.m[2][2]) * hb[2]);
          // (a rounding guard on the scale of the terms: the corner loop rounds its own sums)
          if (!(zlow < off + 1e-6f * (1.0f + fabsf(c.z) + hb[0] + hb[1] + hb[2]))) ty = -1;
        }
      }
      const float* gs = g < G ? mt->gf[g] + 12 : mt->gf[0] + 12;
      int cnt = 0;
      for (int pass = 0; pass < 2; pass++) {
        int k = 0, slot0 = 0;
        if (pass == 1) {
          int tot;
          const int incl = team_scan_bits<T, 9>(cnt, tot);  // a geom's candidates: <= 8, a hull's vertices <= 160
          slot0 = base + incl - cnt;
          base += tot;
        }
        const int nc = ty == MG_GT_SPHERE ? 1 : (ty == MG_GT_CAPSULE ? 2 : (ty == MG_GT_BOX ? 8 : (ty == MG_GT_CONVEX ? mt->hnv : 0)));
        for (int q = 0; q < nc; q++) {
          V3 e;
          float r;
          if (ty == MG_GT_SPHERE) {
            e = c;
            r = gs[0];
          } else if (ty == MG_GT_CAPSULE) {
            V3 ax = v3(Rg.m[0][2], Rg.m[1][2], Rg.m[2][2]) * gs[1];
            e = q == 0 ? c - ax : c + ax;
            r = gs[0];
          } else if (ty == MG_GT_CONVEX) {  // the hull's vertices
            e = c + mul(Rg, ld3(m->hull_vert[q]));
            r = 0.0f;
          } else {
            V3 l = v3((q & 1 ? 1.f : -1.f) * gs[0], (q & 2 ? 1.f : -1.f) * gs[1], (q & 4 ? 1.f : -1.f) * gs[2]);
            e = c + mul(Rg, l);
            r = 0.0f;
          }
          const float d = e.z - r;
          if (!(d < off)) continue;
          if (pass == 0) {
            cnt++;
          } else {
            const int slot = slot0 + k;
            if (slot < cap) put_contact(slot, v3(e.x, e.y, e.z - r), v3(0, 0, 1), d, mt->gnode[g], g, -1, -1);
            k++;
          }
        }
      }
    }
    if constexpr (OBJ != 0) {  // the object on the ground: lane per corner (block), end sphere (pen), or
                               // the egg's support point in -z
      int cnt = 0;
      V3 e = v3(0, 0, 0);
      float r = 0.0f;
      constexpr int ot = OBJ;
      const V3 hb = osize();
      if (ot == MG_GT_BOX && tl < 8) {
        e = mul(oR, v3((tl & 1 ? 1.f : -1.f) * hb.x, (tl & 2 ? 1.f : -1.f) * hb.y, (tl & 4 ? 1.f : -1.f) * hb.z)) + op;
        cnt = 1;
      } else if (ot == MG_GT_CAPSULE && tl < 2) {
        e = mul(oR, v3(0.0f, 0.0f, (tl == 0 ? -1.f : 1.f) * hb.y)) + op;
        r = hb.x;
        cnt = 1;
      } else if (ot == MG_GT_ELLIPSOID && tl == 0) {
        e = mul(oR, ell_support(hb, v3(-oR.m[2][0], -oR.m[2][1], -oR.m[2][2]))) + op;
        cnt = 1;
      }
      const float d = e.z - r;
      cnt = cnt && d < off ? 1 : 0;
      int tot;
      const int incl = team_scan_bits<T, 1>(cnt, tot);
      if (cnt) {
        const int slot = base + incl - 1;
        if (slot < cap) put_contact(slot, v3(e.x, e.y, e.z - r), v3(0, 0, 1), d, OBJ_NODE, -2, -1, -1);
      }
      base += tot;
    }
    ph_mark(19);
    // self-collision pairs, pair order preserved (Humanoid: every non-adjacent pair; ShadowHand: the MJCF's
    // explicit <contact><pair>s).  Pass 1, lane per pair: the bounding-sphere test of the two cores; the
    // survivors' indices are compacted (team scan) into a list in the union storage behind the geom frames.
    // Pass 2, lane per survivor: the segment-segment narrowphase (or segment-box when one side is a box, as
    // the hand's palm against the thumb), so the divergent narrowphase runs over a few dense chunks instead
    // of every chunk of pairs.
    const int P = mt->np;
    const float poff = m->pair_mjcf ? 0.0f : off;  // explicit MJCF pairs: in contact from zero distance (margin 0)
    static_assert(L::kGwFloats >= MG * GW + MP, "the pair list must fit behind the geom frames");
    int* plist = reinterpret_cast<int*>(gw_tile() + GW * MG);
    int npc = 0;
    for (int p0 = 0; p0 < P; p0 += T) {
      const int pi = p0 + tl;
      int ok = 0;
      if (pi < P) {
        // the two geoms' bounding spheres (staged centre, the tile's bounding radius: capsule half length +
        // radius, sphere radius, box half diagonal: the same bound as the cores' spheres); pairs with no segment
        // side have no narrowphase
        const int ga = mt->pairs[pi][0], gb = mt->pairs[pi][1];
        const int ta = mt->gtype[ga], tb2 = mt->gtype[gb];
        const bool sa = ta == MG_GT_SPHERE || ta == MG_GT_CAPSULE, sb = tb2 == MG_GT_SPHERE || tb2 == MG_GT_CAPSULE;
        if (sa || sb) {  // (the non-segment side of a mixed pair is a box: the narrowphase below)
          const V3 dc = ld3(gw_tile() + GW * ga) - ld3(gw_tile() + GW * gb);
          const float reach = mt->gf[ga][15] + mt->gf[gb][15] + poff;
          ok = dot(dc, dc) <= reach * reach ? 1 : 0;
        }
      }
      int scan_tot;
      const int incl = team_scan_bits<T, 1>(ok, scan_tot);
      if (ok) plist[npc + incl - 1] = pi;
      npc += scan_tot;
    }
    wsync();
    static_assert(MP < 256, "wave_max_bits<8>");
    const int npw = wave_max_bits<8>(npc);  // wave-uniform trip count
    for (int c0 = 0; c0 < npw; c0 += T) {
      const int ci = c0 + tl;
      int cnt = 0;
      V3 pt, nrm;
      float d = 0.0f;
      int ga = 0, gb = 0;
      if (ci < npc) {
        const int pi = plist[ci];
        ga = mt->pairs[pi][0];
        gb = mt->pairs[pi][1];
        V3 a0, a1, b0, b1;
        float ra, rb;
        const bool sa = geom_segment(ga, &a0, &a1, &ra), sb = geom_segment(gb, &b0, &b1, &rb);
        if (sa && sb) {
          float ss, tt;
          closest_seg_seg_t(a0, a1, b0, b1, &ss, &tt);
          V3 pa = a0 + (a1 - a0) * ss, pb = b0 + (b1 - b0) * tt, dv = pa - pb;
          float dist = psqrt(dot(dv, dv));
          d = dist - ra - rb;
          if (d < poff && dist > 1e-9f) {
            nrm = dv * prcp(dist);
            pt = ((pa - nrm * ra) + (pb + nrm * rb)) * 0.5f;
            cnt = 1;
          }
        } else {  // box vs sphere / capsule (oracle collide): the segment's closest point to the box
          const int gx = sa ? gb : ga;
          V3 cx;
          M3 Rx;
          geom_staged(gx, &cx, &Rx);
          const float* gs = mt->gf[gx] + 12;
          const V3 hg = v3(gs[0], gs[1], gs[2]);
          const float r = sa ? ra : rb;
          const V3 al = mulT(Rx, (sa ? a0 : b0) - cx), u = mulT(Rx, (sa ? a1 : b1) - cx) - al;
          V3 P, nb, cbx;
          d = seg_box_point(al, u, hg, &P, &nb, &cbx) - r;
          if (d < poff) {
            pt = mul(Rx, ((P - nb * r) + cbx) * 0.5f) + cx;
            nrm = mul(Rx, nb) * (sa ? 1.0f : -1.0f);  // from B to A; nb points from the box to the segment
            cnt = 1;
          }
        }
      }
      int tot;
      const int incl = team_scan_bits<T, 1>(cnt, tot);
      if (cnt) {
        const int slot = base + incl - 1;
        if (slot < cap) put_contact(slot, pt, nrm, d, mt->gnode[ga], ga, mt->gnode[gb], gb);
      }
      base += tot;
    }
    ph_mark(20);
    if constexpr (OBJ != 0) {
      // articulation geoms vs the object: one lane per (geom, candidate) in geom order (the oracle's
      // emission order); a candidate whose geom's bounding sphere cannot come within the contact
      // offset of the object's is skipped (conservative: the same contacts)
      const float ro = obj_radius();
      // pass 1, lane per geom: bounding-sphere cull of the whole geom (its centre only: R . pos + x);
      // the survivors' candidates are then enumerated densely, so culled boxes cost no lanes
      unsigned long long live = 0ull, hull_live = 0ull;
      for (int g0 = 0; g0 < G; g0 += T) {
        const int g = g0 + tl;
        bool ok = false;
        const int gt = g < G ? mt->gtype[g] : -1;
        if (g < G && (mt->gfil[g] & MG_COLLIDE_OBJECT) &&
            (gt == MG_GT_SPHERE || gt == MG_GT_CAPSULE || gt == MG_GT_BOX || gt == MG_GT_CONVEX)) {
          const V3 c = ld3(gw_tile() + GW * g);
          const V3 dc = c - op;
          const float reach = mt->gf[g][15] + ro + off;
          ok = dot(dc, dc) <= reach * reach;
          if (ok && gt == MG_GT_CONVEX) {  // the hull's bounding box against the object's sphere (oracle)
            V3 cc;
            M3 Rg;
            geom_staged(g, &cc, &Rg);
            ok = hull_box_near(cc, Rg, ld3(mt->gf[g] + 12), op, ro, off);
          }
        }
        constexpr unsigned long long tmask = T >= 64 ? ~0ull : ((1ull << T) - 1ull);
        live |= ((__ballot(ok) >> tb) & tmask) << g0;
        hull_live |= ((__ballot(ok && gt == MG_GT_CONVEX) >> tb) & tmask) << g0;
      }
      // the convex-mesh geom first, in a pass of its own (its candidates precede the other geoms' object
      // contacts, as in the oracle's collide; rarely live, and kept out of the main loop's code)
      live &= ~hull_live;
      // block / pen: hull_stage()'s plane bound puts the object at least the contact offset from the hull (every
      // hull candidate's distance is at least that bound), so none of the passes below could emit a contact
      if constexpr (L::HX > 0) {
        if (s->hxn < 0) hull_live = 0ull;
      }
      for (unsigned long long hm = hull_live; hm; hm &= hm - 1) {
        const int g = __builtin_ctzll(hm);
        V3 c;
        M3 Rg;
        geom_staged(g, &c, &Rg);
        // (1) the hull's vertices against the object (block, pen): lane per vertex
        if constexpr (OBJ != MG_GT_ELLIPSOID) {
          const int nhv = mt->hnv;
          for (int f0 = 0; f0 < nhv; f0 += T) {
            const int q = f0 + tl;
            int cnt = 0;
            V3 pt = v3(0, 0, 0), nrm = v3(0, 0, 1);
            float d = 0.0f;
            if (q < nhv) cnt = hull_vertex_candidate(q, c, Rg, &pt, &nrm, &d) && d < off ? 1 : 0;
            int tot;
            const int incl = team_scan_bits<T, 1>(cnt, tot);
            if (cnt) {
              const int slot = base + incl - 1;
              if (slot < cap) put_contact(slot, pt, nrm, d, mt->gnode[g], g, OBJ_NODE, -2);
            }
            base += tot;
          }
        }
        // (2) the object's points against the hull's faces, the faces spread over the team (team argmax;
        // ties -> the lowest face, as the oracle's serial loop): lane k keeps point k's face and distance
        constexpr int K = OBJ == MG_GT_BOX ? 8 : (OBJ == MG_GT_CAPSULE ? 2 : 1);
        const int np = m->hull_num_planes;
        const V3 cl = mulT(Rg, op - c);
        M3 Rl;  // object axes in the geom frame: Rg^T oR
        for (int a = 0; a < 3; a++)
          for (int b = 0; b < 3; b++) Rl.m[a][b] = Rg.m[0][a] * oR.m[0][b] + Rg.m[1][a] * oR.m[1][b] + Rg.m[2][a] * oR.m[2][b];
        float dk = 0.0f;
        int fk = 0;
        if constexpr (OBJ == MG_GT_ELLIPSOID || MG_HULL_FACE_GROUP == 0) {  // (0: round 5's pass per point)
#pragma unroll 1
          for (int k = 0; k < K; k++) {
            const V3 pk = OBJ == MG_GT_ELLIPSOID ? cl : hull_object_point(k, c, Rg);
            float best = -3.0e38f;
            int bf = 0x7fffffff;
            for (int f = tl; f < np; f += T) {
              const float* hp = m->hull_plane[f];
              const V3 x = OBJ == MG_GT_ELLIPSOID ? egg_support_geom(ld3(hp), cl, Rl) : pk;
              const float sd = hp[0] * x.x + hp[1] * x.y + hp[2] * x.z - hp[3];
              if (sd > best) { best = sd; bf = f; }
            }
            team_argmax<T>(best, bf);
            if (tl == k) { dk = best; fk = bf; }
          }
        } else {
          // every object point against each plane the lane loads (one pass over the planes in global memory, the
          // loads of a pass in flight together, instead of one dependent pass per point); per point the same
          // scan order and strict compare, so the same face
          constexpr int KG = K < MG_HULL_FACE_GROUP ? K : (MG_HULL_FACE_GROUP > 0 ? MG_HULL_FACE_GROUP : 1);
#pragma unroll 1
          for (int k0 = 0; k0 < K; k0 += KG) {
            V3 pk[KG];
            float best[KG];
            int bf[KG];
#pragma unroll
            for (int k = 0; k < KG; k++) {
              pk[k] = hull_object_point(k0 + k, c, Rg);
              best[k] = -3.0e38f;
              bf[k] = 0x7fffffff;
            }
            constexpr int NPL = (MG_MAX_HULL_PLANES + T - 1) / T;
#pragma unroll MG_HULL_PLANE_UNROLL
            for (int j = 0; j < NPL; j++) {
              const int f = tl + j * T;
              if (f < np) {
                const float4 q = *reinterpret_cast<const float4*>(m->hull_plane[f]);
#pragma unroll
                for (int k = 0; k < KG; k++) {
                  const float sd = q.x * pk[k].x + q.y * pk[k].y + q.z * pk[k].z - q.w;
                  if (sd > best[k]) { best[k] = sd; bf[k] = f; }
                }
              }
            }
#pragma unroll
            for (int k = 0; k < KG; k++) {
              team_argmax<T>(best[k], bf[k]);
              if (tl == k0 + k) { dk = best[k]; fk = bf[k]; }
            }
          }
        }
        int cnt = 0;
        V3 pt = v3(0, 0, 0), nrm = v3(0, 0, 1);
        float d = 0.0f;
        if (tl < K) {
          const V3 ng = ld3(m->hull_plane[fk]);
          const float ro = OBJ == MG_GT_CAPSULE ? osize().x : 0.0f;
          d = dk - ro;
          const V3 x = OBJ == MG_GT_ELLIPSOID ? egg_support_geom(ng, cl, Rl) : hull_object_point(tl, c, Rg);
          pt = mul(Rg, x - ng * (ro + 0.5f * d)) + c;
          nrm = mul(Rg, ng) * -1.0f;
          cnt = d < off ? 1 : 0;
        }
        int tot;
        const int incl = team_scan_bits<T, 1>(cnt, tot);
        if (cnt) {
          const int slot = base + incl - 1;
          if (slot < cap) put_contact(slot, pt, nrm, d, mt->gnode[g], g, OBJ_NODE, -2);
        }
        base += tot;
        // (3) block / pen: the exact candidates, computed at the start of the substep (hull_stage)
        if constexpr (L::HX > 0) {
          const int nx = s->hxn;
          if (tl < nx && base + tl < cap)
            put_contact(base + tl, ld3(s->hx[tl]), ld3(s->hx[tl] + 3), s->hx[tl][6], mt->gnode[g], g, OBJ_NODE, -2);
          base += nx;
        }
      }
      ph_mark(21);
      // the survivors' candidates in geom order: lane per geom, a team scan of the counts places each geom's
      // run, and the geom writes (geom, candidate index) for its run into a map behind the pair list, so a
      // candidate's lane finds its pair with one LDS read (instead of walking the live mask)
      if constexpr (OBJ == MG_GT_ELLIPSOID) {  // the egg: the candidates egg_stage() computed, in geom order
        const int ne = s->nrows;
        int cnt = 0, g = 0;
        V3 pt = v3(0, 0, 0), nrm = v3(0, 0, 1);
        float d = 0.0f;
        if (tl < ne) {
          pt = ld3(s->ct1[tl]);
          nrm = ld3(s->ct2[tl]);
          d = __int_as_float(s->lmeta[tl]);
          g = s->lmeta[MN - 1 + tl];
          cnt = d < off ? 1 : 0;
        }
        int tot;
        const int incl = team_scan_bits<T, 1>(cnt, tot);
        if (cnt) {
          const int slot = base + incl - 1;
          if (slot < cap) put_contact(slot, pt, nrm, d, mt->gnode[g], g, OBJ_NODE, -2);
        }
        base += tot;
      } else {
      static_assert(L::kGwFloats >= MG * GW + MP + (17 * MG + 1) / 2, "the candidate map must fit behind the pair list");
      uint16_t* cmap = reinterpret_cast<uint16_t*>(plist + MP);
      int NC = 0;
      for (int g0 = 0; g0 < G; g0 += T) {
        const int g = g0 + tl;
        const int n = (g < G && ((live >> g) & 1ull)) ? ocand_count(mt->gtype[g]) : 0;
        int tot;
        const int incl = team_scan_bits<T, 9>(n, tot);  // a geom's object candidates (the hull's planes: <= 320)
        for (int q = 0; q < n; q++) cmap[NC + incl - n + q] = (uint16_t)(g | (q << 8));
        NC += tot;
      }
      wsync();
      for (int f0 = 0; f0 < NC; f0 += T) {
        const int f = f0 + tl;
        int cnt = 0, g = 0;
        V3 pt = v3(0, 0, 0), nrm = v3(0, 0, 1);
        float d = 0.0f;
        if (f < NC) {
          const int e = cmap[f];
          g = e & 0xff;
          const int q = e >> 8;
          V3 c;
          M3 Rg;
          geom_staged(g, &c, &Rg);
          bool ok;
          if constexpr (OBJ == MG_GT_BOX) ok = obj_candidate(g, q, c, Rg, &pt, &nrm, &d);
          else ok = obj_candidate_convex(g, q, c, Rg, &pt, &nrm, &d);
          cnt = ok && d < off ? 1 : 0;
        }
        int tot;
        const int incl = team_scan_bits<T, 1>(cnt, tot);
        if (cnt) {
          const int slot = base + incl - 1;
          if (slot < cap) put_contact(slot, pt, nrm, d, mt->gnode[g], g, OBJ_NODE, -2);
        }
        base += tot;
      }
      }
    }
    if (tl == 0) s->ncon = base < cap ? base : cap;
    wsync();
  }

  static __device__ void closest_seg_seg_t(V3 p1, V3 q1, V3 p2, V3 q2, float* s_out, float* t_out) {
    V3 d1 = q1 - p1, d2 = q2 - p2, r = p1 - p2;
    float a = dot(d1, d1), e = dot(d2, d2), f = dot(d2, r);
    float sv_, tv;
    const float eps = 1e-12f;
    if (a <= eps && e <= eps) {
      sv_ = tv = 0;
    } else if (a <= eps) {
      sv_ = 0;
      tv = fminf(fmaxf(f * prcp(e), 0.0f), 1.0f);
    } else {
      float c = dot(d1, r);
      if (e <= eps) {
        tv = 0;
        sv_ = fminf(fmaxf(-c * prcp(a), 0.0f), 1.0f);
      } else {
        float b = dot(d1, d2), den = a * e - b * b;
        const float ia = prcp(a), ie = prcp(e);
        sv_ = den > eps ? (b * f - c * e) * prcp(den) : 0.0f;
        sv_ = fminf(fmaxf(sv_, 0.0f), 1.0f);
        tv = (b * sv_ + f) * ie;
        if (tv < 0) {
          tv = 0;
          sv_ = fminf(fmaxf(-c * ia, 0.0f), 1.0f);
        } else if (tv > 1) {
          tv = 1;
          sv_ = fminf(fmaxf((b - c) * ia, 0.0f), 1.0f);
        }
      }
    }
    *s_out = sv_;
    *t_out = tv;
  }

  // ---------------------------------------------------------------- constraint rows
  __device__ __forceinline__ void build_rows() {
    const int ncon = ncr;
    const float ih = prcp(h);
    for (int c = tl; c < ncon; c += T) {
      V3 n = ld3(s->cn[c]), pt = ld3(s->cp[c]), t1, t2;
      tangent_basis_t(n, &t1, &t2);
      s->set_tangents(c, t1, t2);
      float deff = s->gap(c) - p->rest_offset;
      float bn = deff >= 0.0f ? -deff * ih : fminf(-p->baumgarte * deff * ih, p->max_depen_vel);
      s->rows()[3 * c].b = TGS ? deff : bn;   // TGS: the gap; its target is set per sweep (substep())
      s->rows()[3 * c + 1].b = 0.0f;
      s->rows()[3 * c + 2].b = 0.0f;
      if constexpr (L::OROWS > 1) {  // the object's columns [w; v_com]: +-[(p - c_obj) x d; d]
        const float so = (cside(c, 0) == OBJ_NODE ? 1.0f : 0.0f) - (cside(c, 1) == OBJ_NODE ? 1.0f : 0.0f);
        V3 dirs[3] = {n, t1, t2};
        for (int r = 0; r < 3; r++) {
          const int row = 3 * c + r;
          const V3 wo = cross(pt - op, dirs[r]) * so, d = dirs[r] * so;
          s->rwo[row][0] = wo.x; s->rwo[row][1] = wo.y; s->rwo[row][2] = wo.z;
          s->rwo[row][3] = d.x; s->rwo[row][4] = d.y; s->rwo[row][5] = d.z;
        }
      }
    }
    // joint-limit rows in DOF order (lower, then upper)
    int cnt = 0;
    float dl = 0.0f, du = 0.0f;
    bool lo = false, hi = false;
    if (node > 0 && mt->limited[node]) {
      const float* np = nprop(node);
      dl = qj - np[4];
      du = np[5] - qj;
      lo = dl < p->limit_margin;
      hi = du < p->limit_margin;
      cnt = (lo ? 1 : 0) + (hi ? 1 : 0);
    }
    int tot;
    const int incl = team_scan_bits<T, 2>(cnt, tot);
    int li = incl - cnt;
    sat = (sat & 1) | (lo ? 2 : 0) | (hi ? 4 : 0) | (li << 3);
    for (int side = 0; side < 2; side++) {
      bool on = side == 0 ? lo : hi;
      if (!on) continue;
      float d = side == 0 ? dl : du;
      s->rows()[3 * ncon + li].b = TGS ? d : (d >= 0.0f ? -d * ih : fminf(-p->baumgarte * d * ih, p->max_depen_vel));
      s->set_lm(li, (2 + side) | (node << 4));
      li++;
    }
    if (tl == 0) s->nrows = 3 * ncon + tot;
    wsync();
  }

  // the root coupling Wv of the test solves (substep()) from the root inverse aba() left in Iinv
  __device__ __forceinline__ void root_coupling(float* Wv) const {
    if (!freeb) return;
    if (tl < 6) {
      for (int k = 0; k < 6; k++) Wv[k] = -s->iinv()[6 * tl + k];
    } else if (node > 0) {
      const float Uv[6] = {U.a.x, U.a.y, U.a.z, U.l.x, U.l.y, U.l.z};
      for (int k = 0; k < 6; k++) {
        float w = 0.0f;
        for (int c2 = 0; c2 < 6; c2++) w += s->iinv()[6 * c2 + k] * Uv[c2];
        Wv[k] = w;
      }
    }
  }

  // ---------------------------------------------------------------- one substep
  __device__ __forceinline__ void substep() {
    ph_mark(15);
    hull_stage();
    ph_mark(22);
    fk();
    if constexpr (OBJ == MG_GT_ELLIPSOID) {
      egg_stage();
      reload_tree();
    }
    set_axis();
    ph_mark(0);
    if (OBJ) tendons();
    aba();
    // root coupling of the test solves: with a0 = -IA0^-1 p0, a joint lane's U.a0 = -(IA0^-1 U).p0
    // and a root lane's a0[tl] = -(row tl of IA0^-1).p0, so one 6-vector per lane covers both.  The compact
    // layout takes it now (its Iinv shares region B with collide()'s geom frames), the other after build_rows()
    float Wv[6] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    if constexpr (L::kCompact) root_coupling(Wv);
    ph_mark(1);
    obj_free();
    collide();
    ncr = s->ncon;
    if constexpr (L::kCompact) org = p0;  // the bits fk() stored in x[0]: region A holds the gaps by now
    else org = ld3(s->x[0]);
    ph_mark(2);
    build_rows();
    ph_mark(3);
    const int nrows = s->nrows;
    static_assert(MR < 256, "wave_max_bits<8>");
    const int wave_rows = wave_max_bits<8>(nrows);
#ifdef MG_PHASE_TIMING
    ph[13] += wave_rows;
#endif
    // row responses Y_r = M~^-1 J_r^T by test-force ABA solves (column distributed over the lanes),
    // W_r = J_r . Y_r.  Lane j keeps (J_r[j], Y_r[j]) of every row in private arrays for the sweeps;
    // rows past this team's count get J = Y = 0 and zero scalars, so the sweeps need no row mask.
    if constexpr (!L::kCompact) {
      if (wave_rows > 0) root_coupling(Wv);
    }
    // (J_r[j], Y_r[j]) of the first KR rows live in registers (the index is wave-uniform, so the compiler
    // promotes the arrays to VGPRs and addresses them with relative moves); the remaining rows are
    // private arrays in scratch.  Wave-uniform branches pick the side.
#if MG_PART_B_LDS
    constexpr int KR = L::KR, PBL = L::PBL;
    float Jr[KR > 0 ? KR : 1], Yr[KR > 0 ? KR : 1];
    float Js[MR - KR - PBL > 0 ? MR - KR - PBL : 1], Ys[MR - KR - PBL > 0 ? MR - KR - PBL : 1];
    // part B: rows KR .. KR + PBL - 1 in the dead tree tiles (J rows, then Y rows, lane-contiguous), the rest scratch
    float* const pbj = &s->R[1][0] + tl;
    float* const pby = pbj + PBL * T;
#define MG_JSET(r, j, y)                                   \
  do {                                                     \
    if ((r) < KR) {                                        \
      Jr[r] = (j); Yr[r] = (y);                            \
    } else if ((r) < KR + PBL) {                           \
      pbj[((r) - KR) * T] = (j); pby[((r) - KR) * T] = (y); \
    } else {                                               \
      Js[(r) - KR - PBL] = (j); Ys[(r) - KR - PBL] = (y);   \
    }                                                      \
  } while (0)
#define MG_JGET(r, jo, yo)                                     \
  do {                                                         \
    if ((r) < KR + PBL) {                                      \
      jo = pbj[((r) - KR) * T]; yo = pby[((r) - KR) * T];      \
    } else {                                                   \
      jo = Js[(r) - KR - PBL]; yo = Ys[(r) - KR - PBL];        \
    }                                                          \
  } while (0)
#else
    constexpr int KR = L::KR;
    float Jr[KR > 0 ? KR : 1], Yr[KR > 0 ? KR : 1];
    float Js[MR - KR > 0 ? MR - KR : 1], Ys[MR - KR > 0 ? MR - KR : 1];
#define MG_JSET(r, j, y)                 \
  do {                                   \
    if ((r) < KR) {                      \
      Jr[r] = (j); Yr[r] = (y);          \
    } else {                             \
      Js[(r) - KR] = (j); Ys[(r) - KR] = (y); \
    }                                    \
  } while (0)
#define MG_JGET(r, jo, yo)               \
  do {                                   \
    jo = Js[(r) - KR]; yo = Ys[(r) - KR]; \
  } while (0)
#endif
    for (int r0 = 0; r0 < wave_rows; r0 += L::RB) {
      float jb[L::RB], yb[L::RB];
#pragma unroll
      for (int g = 0; g < L::RB; g += 3) batch_jacobians(r0 + g, nrows, jb + g);
      ph_mark(4);
      test_solve(r0, nrows, Wv, yb);
      // the row record of row r (written by one lane): 1/W, impulse 0, mu; inactive rows get b = 0
      auto row_record = [&](int r, float Wr) {
        const bool active = r < nrows;
        const bool contact = r < 3 * ncr;
        typename L::Row& rw = s->rows()[r];
        rw.iw = (active && Wr > 1e-12f) ? prcp(Wr) : 0.0f;
        rw.lam = 0.0f;
        // DR: a contact's friction is the mean of its two shapes' (vec_task.py rigid_shape_properties)
        float muc = (drg && contact) ? 0.5f * (gmu(cside(r / 3, 2)) + gmu(cside(r / 3, 3))) : p->friction;
        if (contact && m->pair_mjcf && cside(r / 3, 1) >= 0) muc = 0.0f;  // explicit MJCF pair: condim 1
        rw.mu = contact ? (r % 3 == 0 ? -1.0f : muc) : -2.0f;
        if (!active) rw.b = 0.0f;
      };
      float wq[L::RB];
#pragma unroll
      for (int q = 0; q < L::RB; q++) {
        const int r = r0 + q;
        wq[q] = 0.0f;
        if (r < wave_rows) {
          const bool active = r < nrows;
          const bool contact = r < 3 * ncr;
          float y = yb[q];
          if (OBJ && objl) y = contact ? obj_response(r) : 0.0f;
          y = active ? y : 0.0f;
          const float J = jb[q];
          MG_JSET(r, J, y);
          const float Wr = team_sum<T>(J * y, tb);
          wq[q] = Wr;
        }
      }
      {  // the block's row records, lane q writes row r0 + q: one divergent region instead of RB
        float Wr = wq[0];
#pragma unroll
        for (int q = 1; q < L::RB; q++) Wr = tl == q ? wq[q] : Wr;
        if (tl < L::RB && r0 + tl < wave_rows) row_record(r0 + tl, Wr);
      }
      ph_mark(5);
    }
    // The sweep runs over prow rows, the row count rounded up to a multiple of the prefetch depth PF
    // (so a row's impulse is never read ahead of its previous visit's write, and the unrolled loop
    // needs no per-visit guards): the padding rows have J = Y = 0 and 1/W = 0, i.e. they are skipped
    // as the oracle skips W = 0 rows.
    drop_tree_state();
    constexpr int PF = kPgsPrefetch;
    static_assert(MR % PF == 0, "row capacity must be a multiple of the PGS prefetch depth");
    const int prow = wave_rows == 0 ? 0 : ((wave_rows + PF - 1) / PF) * PF;
    for (int r = wave_rows; r < prow; r++) MG_JSET(r, 0.0f, 0.0f);
    if (tl < prow - wave_rows) s->rows()[wave_rows + tl] = typename L::Row{0.0f, 0.0f, 0.0f, -2.0f};  // PF - 1 <= T
    wsync();
    ph_mark(5);
    // PGS sweeps: per visit one team dot product (DPP), a branch-free clamp (med3), one multiply-add
    // per lane.  A visit's data (private J/Y, LDS row record) do not depend on the sweep's chain; they
    // sit in PF rotating registers loaded PF visits ahead, each load issued after the previous
    // occupant's last use.  The friction bound uses the contact's normal impulse of this sweep (the
    // normal row precedes its two friction rows), carried in a register.  Every lane of the team
    // computes the same impulse, so all of them store it (no exec-mask switch per visit).
    // Rows below KR take their (J, Y) from registers in a fully unrolled part A (static indices; the LDS
    // row records are loaded one block ahead); the rows from KR on run part B, whose scratch columns and
    // row records rotate through PF registers loaded a block ahead and wrap into the next sweep's part B.
    float lamn = 0.0f;
    // TGS: the sub-steps' accumulated displacement of this lane's column, 1 / (h / N), and the sweeps: N position
    // sub-steps, then max(N, vel_iters) velocity sweeps with the bias off (a separated row's speculative target on h)
    float dqs = 0.0f;
    const float hs = TGS ? h / (float)(p->pos_iters > 0 ? p->pos_iters : 1) : 0.0f;
    const float ihs = TGS ? prcp(hs) : 0.0f;
    float tisp = ihs, tbz = TGS ? p->baumgarte : 0.0f;
    const int n_sweeps = TGS ? p->pos_iters + max(p->pos_iters, p->vel_iters) : p->pos_iters;
    auto visit = [&](float J, float Y, const typename L::Row& R, int r) {
      MG_NC_PGS
      const float v = team_sum<T>(J * nu, tb);
      const float lam = R.lam, m = R.mu;
      // friction rows (m = mu >= 0): [-mu lambda_n, mu lambda_n]; normal / limit rows (m < 0):
      // [0, inf).  Rows with 1/W = 0 keep lambda = 0: lam + (b - v) * 0 = 0 clamps to 0.
      const bool fric = m >= 0.0f;
      const float t = fric ? m * lamn : 0.0f;
      const float hi = fric ? t : __builtin_inff();
      float tgt = R.b;
      if constexpr (TGS) {  // target from the gap moved by the sub-steps so far: e = e0 + J . dq, on h / N
        const float e = R.b + team_sum<T>(J * dqs, tb);
        const float te = e >= 0.0f ? -e * tisp : fminf(-tbz * e * ihs, p->max_depen_vel);
        tgt = fric ? 0.0f : te;
      }
#if MG_PGS_UNFUSE & 2
      float dlr = (tgt - v) * R.iw;
      asm volatile("" : "+v"(dlr));  // (A/B: the impulse update's product rounded, not fused)
      const float lnew = __builtin_amdgcn_fmed3f(lam + dlr, -t, hi);
#else
      const float lnew = __builtin_amdgcn_fmed3f(lam + (tgt - v) * R.iw, -t, hi);
#endif
      lamn = m == -1.0f ? lnew : lamn;
      s->rows()[r].lam = lnew;
#if MG_PGS_UNFUSE & 1
      float dv = Y * (lnew - lam);
      asm volatile("" : "+v"(dv));  // (A/B: the velocity update's product rounded, not fused)
      nu += dv;
#else
      nu += Y * (lnew - lam);
#endif
    };
    const int pa = prow < KR ? prow : KR;  // rows of part A
    float pJ[PF], pY[PF];
    typename L::Row pR[PF];
    if (prow > KR) {
#pragma unroll
      for (int k = 0; k < PF; k++) {
        MG_JGET(KR + k, pJ[k], pY[k]);
        pR[k] = s->rows()[KR + k];
      }
    }
    for (int it = 0; it < n_sweeps; it++) {
      if constexpr (TGS) {
        if (it == p->pos_iters) {  // the velocity sweeps: bias off
          tisp = prcp(h);
          tbz = 0.0f;
        }
      }
      if constexpr (KR > 0) {
        typename L::Row cR[PF];
        if (pa > 0) {
#pragma unroll
          for (int k = 0; k < PF; k++) cR[k] = s->rows()[k];
        }
#pragma unroll
        for (int r0 = 0; r0 < KR; r0 += PF) {
          if (r0 < pa) {
            typename L::Row nR[PF];
            const bool more = r0 + PF < pa;
            if (more) {
#pragma unroll
              for (int k = 0; k < PF; k++) nR[k] = s->rows()[r0 + PF + k];
            }
#pragma unroll
            for (int k = 0; k < PF; k++) visit(Jr[r0 + k], Yr[r0 + k], cR[k], r0 + k);
            if (more) {
#pragma unroll
              for (int k = 0; k < PF; k++) cR[k] = nR[k];
            }
          }
        }
      }
      for (int r0 = KR; r0 < prow; r0 += PF) {
        const int rn = r0 + PF == prow ? KR : r0 + PF;  // next block of part B (wraps into the next sweep)
        // the next block's private J/Y (scratch, L2 latency) are issued before this block's visits; the
        // compiler barrier keeps the scheduler from sinking them behind the first visits
        float nJ[PF], nY[PF];
#pragma unroll
        for (int k = 0; k < PF; k++) MG_JGET(rn + k, nJ[k], nY[k]);
        asm volatile("" ::: "memory");
#pragma unroll
        for (int k = 0; k < PF; k++) {
          visit(pJ[k], pY[k], pR[k], r0 + k);
          pJ[k] = nJ[k];
          pY[k] = nY[k];
          pR[k] = s->rows()[rn + k];
        }
      }
      if constexpr (TGS) {  // the sub-step's displacement
        if (it < p->pos_iters) dqs += hs * nu;
      }
    }
    wsync();
#undef MG_JSET
#undef MG_JGET
    ph_mark(6);
    clamp_ang_vel();
    if constexpr (TGS) {
      integrate_tgs(dqs);
    } else {
      integrate();
    }
    ph_mark(7);
  }

  // The tree phases assign R, x, S, V, c, U, pA, IA, D^-1, u only on the lanes of the level being
  // processed, so without help the compiler keeps every lane's previous value alive across the whole
  // substep loop.  None is read again before the next substep's fk()/aba() rewrite them (outputs()
  // reruns fk()), so they are set to constants once the rows are built: their registers are free
  // for the PGS sweep.
  __device__ __forceinline__ void drop_tree_state() {
    R = M3{};
    x = v3(0, 0, 0);
    S = V = c = U = pA = szero();
    IA = Sym6{};
    Dinv = u = 0.0f;
    for (int k = 0; k < 6; k++) Sl[k] = 0.0f;
  }

  // gym AssetOptions.max_angular_velocity (humanoid.py:154; gym default 64, the object's too): after the solve
  // every link's |w| <= W.  Root first (w scaled to W, its COM velocity kept); then level by level each hinge's
  // rate is clamped to { t : |w_parent + a t| <= W } (a = its unit world axis, s->S from this substep's fk),
  // which holds t = 0 because the parent is clamped already; slides carry the parent's w.  Same rule as the
  // oracle's clamp_ang_vel.  A team bound |w_root| + sum |qd| <= W (no link can reach the cap) skips the pass.
  __device__ __forceinline__ void clamp_ang_vel() {
    MG_NC_INT
    const float W = m->link_max_ang_vel;
    if (W > 0.0f) {
      const V3 w0 = freeb ? v3(__shfl(nu, tb), __shfl(nu, tb + 1), __shfl(nu, tb + 2)) : v3(0, 0, 0);
      const bool hinge = node > 0 && mt->jtype[node] == MG_JT_HINGE;
      const float n0 = sqrtf(dot(w0, w0));
      const float bound = n0 + team_sum<T>(hinge ? fabsf(nu) : 0.0f, tb);
      if (__ballot(bound > W) != 0ull) {  // wave-uniform
        V3 wr = w0;
        if (freeb && n0 > W) {
          wr = w0 * (W / n0);
          if (tl < 3) {
            nu = tl == 0 ? wr.x : (tl == 1 ? wr.y : wr.z);
          } else if (tl < 6) {
            M3 Rr;  // fk()'s R[0] (compact: region A holds the rows; quat_to_mat(q0) gives the same bits)
            if constexpr (L::kCompact) {
              Rr = quat_to_mat(q0[0], q0[1], q0[2], q0[3]);
            } else {
              for (int a = 0; a < 3; a++)
                for (int b = 0; b < 3; b++) Rr.m[a][b] = s->R[0][3 * a + b];
            }
            const V3 dv = cross(w0 - wr, mul(Rr, ld3(m->body_com[0])));
            nu += tl == 3 ? dv.x : (tl == 4 ? dv.y : dv.z);
          }
        }
        V3 om = wr;
        const V3 ax = node > 0 ? ld3(s->S[node]) : v3(0, 0, 0);
        const int pl = tb + (par > 0 ? col_of(par) : 0);
        for (int lev = 1; lev <= maxdepth; lev++) {
          const V3 wl = v3(__shfl(om.x, pl), __shfl(om.y, pl), __shfl(om.z, pl));
          if (node > 0 && depth == lev) {
            const V3 wp = par > 0 ? wl : wr;
            if (hinge) {
              V3 w = wp + ax * nu;
              if (dot(w, w) > W * W) {
                const float b = dot(ax, wp);
                const float sq = sqrtf(fmaxf(b * b - dot(wp, wp) + W * W, 0.0f));
                nu = fminf(fmaxf(nu, -b - sq), -b + sq);
                w = wp + ax * nu;
              }
              om = w;
            } else {
              om = wp;
            }
          }
        }
      }
    }
    if (OBJ && m->obj_max_ang_vel > 0.0f) {
      const V3 w = v3(__shfl(nu, tb + ob0), __shfl(nu, tb + ob0 + 1), __shfl(nu, tb + ob0 + 2));
      const float n = sqrtf(dot(w, w));
      if (objl && tl - ob0 < 3 && n > m->obj_max_ang_vel) nu *= m->obj_max_ang_vel / n;
    }
  }

  __device__ __forceinline__ void integrate() {
    MG_NC_INT
    // root pose (lane 0 gathers the twist from lanes 0..5)
    float w0 = __shfl(nu, tb + 0), w1 = __shfl(nu, tb + 1), w2 = __shfl(nu, tb + 2);
    float v0 = __shfl(nu, tb + 3), v1 = __shfl(nu, tb + 4), v2 = __shfl(nu, tb + 5);
    if (freeb) {
      V3 om = v3(w0, w1, w2), vo = v3(v0, v1, v2);
      V3 pn = p0 + vo * h;
      float wn = sqrtf(dot(om, om));
      float dq[4];
      if (wn * h > 1e-12f) {
        float sh, ch;
        psincos<kHwTrig>(0.5f * wn * h, &sh, &ch);
        const float sn = sh * prcp(wn);
        dq[0] = om.x * sn; dq[1] = om.y * sn; dq[2] = om.z * sn; dq[3] = ch;
      } else {
        dq[0] = 0.5f * h * om.x; dq[1] = 0.5f * h * om.y; dq[2] = 0.5f * h * om.z; dq[3] = 1.0f;
      }
      const float* a = dq;
      const float* b = q0;
      float qn[4] = {a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1],
                     a[3] * b[1] - a[0] * b[2] + a[1] * b[3] + a[2] * b[0],
                     a[3] * b[2] + a[0] * b[1] - a[1] * b[0] + a[2] * b[3],
                     a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2]};
      float l = prsq(qn[0] * qn[0] + qn[1] * qn[1] + qn[2] * qn[2] + qn[3] * qn[3]);
      for (int k = 0; k < 4; k++) q0[k] = qn[k] * l;
      V3 dp = pn - p0;
      p0 = pn;
      V3 vn = vo + cross(om, dp);
      if (tl == 3) nu = vn.x;
      if (tl == 4) nu = vn.y;
      if (tl == 5) nu = vn.z;
    }
    if (node > 0) qj += h * nu;
    if (OBJ) {  // free object: pose replicated on every lane (exponential map, like the root)
      const V3 om = v3(__shfl(nu, tb + ob0), __shfl(nu, tb + ob0 + 1), __shfl(nu, tb + ob0 + 2));
      const V3 vc = v3(__shfl(nu, tb + ob0 + 3), __shfl(nu, tb + ob0 + 4), __shfl(nu, tb + ob0 + 5));
      const float wn = sqrtf(dot(om, om));
      float dq[4];
      if (wn * h > 1e-12f) {
        const float ha = 0.5f * wn * h, sn = sinf(ha) * prcp(wn);
        dq[0] = om.x * sn; dq[1] = om.y * sn; dq[2] = om.z * sn; dq[3] = cosf(ha);
      } else {
        dq[0] = 0.5f * h * om.x; dq[1] = 0.5f * h * om.y; dq[2] = 0.5f * h * om.z; dq[3] = 1.0f;
      }
      const float* a = dq;
      const float* b = oq;
      float qn[4] = {a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1],
                     a[3] * b[1] - a[0] * b[2] + a[1] * b[3] + a[2] * b[0],
                     a[3] * b[2] + a[0] * b[1] - a[1] * b[0] + a[2] * b[3],
                     a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2]};
      const float l = prsq(qn[0] * qn[0] + qn[1] * qn[1] + qn[2] * qn[2] + qn[3] * qn[3]);
      for (int k = 0; k < 4; k++) oq[k] = qn[k] * l;
      op = op + vc * h;
    }
  }

  // TGS: positions by the sub-steps' accumulated displacement dq (this lane's column) instead of h nu -- the root's
  // rotation vector dq[0..2] by the exponential map, its origin by dq[3..5], the final twist re-expressed at the new
  // origin; joints q += dq; the free object likewise; velocities are the final nu, after the velocity sweeps and the
  // cap (oracle tgs_integrate).
  __device__ __forceinline__ static void rotvec_quat(V3 th, float* q) {
    const float tn = sqrtf(dot(th, th));
    float d[4];
    if (tn > 1e-12f) {
      const float ha = 0.5f * tn, sn = sinf(ha) * prcp(tn);
      d[0] = th.x * sn; d[1] = th.y * sn; d[2] = th.z * sn; d[3] = cosf(ha);
    } else {
      d[0] = 0.5f * th.x; d[1] = 0.5f * th.y; d[2] = 0.5f * th.z; d[3] = 1.0f;
    }
    const float* a = d;
    const float b[4] = {q[0], q[1], q[2], q[3]};
    float qn[4] = {a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1],
                   a[3] * b[1] - a[0] * b[2] + a[1] * b[3] + a[2] * b[0],
                   a[3] * b[2] + a[0] * b[1] - a[1] * b[0] + a[2] * b[3],
                   a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2]};
    const float l = prsq(qn[0] * qn[0] + qn[1] * qn[1] + qn[2] * qn[2] + qn[3] * qn[3]);
    for (int k = 0; k < 4; k++) q[k] = qn[k] * l;
  }
  __device__ __forceinline__ void integrate_tgs(float dq) {
    if (freeb) {
      const V3 th = v3(__shfl(dq, tb + 0), __shfl(dq, tb + 1), __shfl(dq, tb + 2));
      const V3 dp = v3(__shfl(dq, tb + 3), __shfl(dq, tb + 4), __shfl(dq, tb + 5));
      const V3 om = v3(__shfl(nu, tb + 0), __shfl(nu, tb + 1), __shfl(nu, tb + 2));
      const V3 vo = v3(__shfl(nu, tb + 3), __shfl(nu, tb + 4), __shfl(nu, tb + 5));
      rotvec_quat(th, q0);
      p0 = p0 + dp;
      const V3 vn = vo + cross(om, dp);
      if (tl == 3) nu = vn.x;
      if (tl == 4) nu = vn.y;
      if (tl == 5) nu = vn.z;
    }
    if (node > 0) qj += dq;
    if (OBJ) {
      const V3 th = v3(__shfl(dq, tb + ob0), __shfl(dq, tb + ob0 + 1), __shfl(dq, tb + ob0 + 2));
      const V3 dp = v3(__shfl(dq, tb + ob0 + 3), __shfl(dq, tb + ob0 + 4), __shfl(dq, tb + ob0 + 5));
      rotvec_quat(th, oq);
      op = op + dp;
    }
  }

  // ---------------------------------------------------------------- sensors & DOF forces (last substep)
  // Sensor wrenches lane-parallel over the contacts (wide locomotion teams: Humanoid's 2 sensors against up to
  // 32 contacts).  Contact c sits on lane c mod T: its impulse as a world force f_c and the bodies of its two
  // sides (+ side A, - side B, A first, as the per-sensor scan).  Sensor k's wrench about its body origin x_k is
  // the team sum of +-[f_c; (p_c - x_k) x f_c]; the six sums of a sensor are independent, so a sensor costs a
  // few pipelined reductions instead of a serial scan over the contacts.  The sensor tables are read with
  // wave-uniform indices (scalar loads).  Same-box A/B: Humanoid +1.1 %; Ant -1.3 % and ShadowHand -0.9 %
  // (4-5 sensors against a handful of contacts), which keep the scan.
  __device__ __forceinline__ void sensors_by_team_sums(float* sens_out, int NS) {
    constexpr int CPL = (MC + T - 1) / T;  // contacts per lane
    const int nc = s->ncon;
    V3 f[CPL], pc[CPL];
    int ba[CPL], bb[CPL];
#pragma unroll
    for (int j = 0; j < CPL; j++) {
      const int c = tl + j * T;
      f[j] = v3(0, 0, 0);
      pc[j] = v3(0, 0, 0);
      ba[j] = bb[j] = -1;
      if (c < nc) {
        const int ga = cside(c, 2), gb = cside(c, 3);
        ba[j] = ga >= 0 ? mt->gbody[ga] : -1;
        bb[j] = gb >= 0 ? mt->gbody[gb] : -1;
        if constexpr (L::kCompact) {  // the impulse sum outputs() stashed before its fk() overwrote the rows
          f[j] = ld3(s->fc(c)) * prcp(h);
        } else {
          const V3 n = ld3(s->cn[c]);
          V3 t1, t2;
          s->tangents(c, &t1, &t2);  // build_rows' basis
          f[j] = (n * s->rows()[3 * c].lam + t1 * s->rows()[3 * c + 1].lam + t2 * s->rows()[3 * c + 2].lam) *
                 prcp(h);
        }
        pc[j] = ld3(s->cp[c]);
      }
    }
    V3 F = v3(0, 0, 0), Tq = v3(0, 0, 0);
    M3 Rb;
#pragma unroll
    for (int k = 0; k < MG_MAX_SENSORS; k++) {
      if (k >= NS) break;  // wave-uniform
      const int body = m->sensor_body[k], nd = m->body_node[body];
      M3 Rn;
      for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) Rn.m[a][b] = s->R[nd][3 * a + b];
      const V3 xb = ld3(s->x[nd]) + mul(Rn, ld3(m->body_pos[body]));
      V3 fs = v3(0, 0, 0), ts = v3(0, 0, 0);
#pragma unroll
      for (int j = 0; j < CPL; j++) {
        const float sg = ba[j] == body ? 1.0f : (bb[j] == body ? -1.0f : 0.0f);
        const V3 fk = f[j] * sg;
        fs = fs + fk;
        ts = ts + cross(pc[j] - xb, fk);
      }
      const float s0 = team_sum<T>(fs.x, tb), s1 = team_sum<T>(fs.y, tb), s2 = team_sum<T>(fs.z, tb);
      const float s3 = team_sum<T>(ts.x, tb), s4 = team_sum<T>(ts.y, tb), s5 = team_sum<T>(ts.z, tb);
      if (tl == k) {
        F = v3(s0, s1, s2);
        Tq = v3(s3, s4, s5);
        Rb = mul(Rn, quat_to_mat(m->body_quat[body][0], m->body_quat[body][1], m->body_quat[body][2],
                                 m->body_quat[body][3]));
      }
    }
    if (tl < NS) {
      const V3 Fl = mulT(Rb, F), Tl = mulT(Rb, Tq);
      float* o = sens_out + 6 * tl;
      o[0] = Fl.x; o[1] = Fl.y; o[2] = Fl.z; o[3] = Tl.x; o[4] = Tl.y; o[5] = Tl.z;
    }
  }
  // POSE: the caller reads no link velocity / axis afterwards (k_env_step; k_simulate and k_hand_step write the
  // rigid-body states from them)
  // ncf_out: this actor's rows of the net contact force tensor (mg_state_views.net_contact_forces), or nullptr
  template <bool POSE = false>
  __device__ __forceinline__ void outputs(float* sens_out, float* dforce_out, float* ncf_out = nullptr) {
    // the compact layout keeps the last substep's rows in region A, which fk() overwrites: each contact's impulse
    // sum goes to region B (fc) and a node's limit impulses to registers first
    float llo = 0.0f, lhi = 0.0f;
    if constexpr (L::kCompact) {
      const int nc = s->ncon;
      for (int c = tl; c < nc; c += T) {
        const V3 n = ld3(s->cn[c]);
        V3 t1, t2;
        s->tangents(c, &t1, &t2);  // build_rows' basis
        const V3 f = n * s->rows()[3 * c].lam + t1 * s->rows()[3 * c + 1].lam + t2 * s->rows()[3 * c + 2].lam;
        float* o = s->fc(c);
        o[0] = f.x; o[1] = f.y; o[2] = f.z;
      }
      if (node > 0) {
        const int lr = 3 * nc + (sat >> 3);
        if (sat & 2) llo = s->rows()[lr].lam;
        if (sat & 4) lhi = s->rows()[lr + ((sat >> 1) & 1)].lam;
      }
      wsync();
    }
    // net contact forces (gym acquire_net_contact_force_tensor): lane per body (articulation bodies, then the object
    // and the goal), the contacts in order as the oracle's net_contact_forces sums them: + on side A, - on side B
    if (ncf_out) {
      const int nb = m->num_bodies, nbe = nb + (OBJ ? 2 : 0), nc = s->ncon;
      const float ihc = prcp(h);
      for (int b = tl; b < nbe; b += T) {
        V3 F = v3(0, 0, 0);
        for (int c = 0; c < nc; c++) {
          const int gA = cside(c, 2), gB = cside(c, 3);
          const int bA = gA >= 0 ? mt->gbody[gA] : (gA == -2 ? nb : -1), bB = gB >= 0 ? mt->gbody[gB] : (gB == -2 ? nb : -1);
          if (bA != b && bB != b) continue;
          V3 f;
          if constexpr (L::kCompact) {
            f = ld3(s->fc(c));
          } else {
            const V3 n = ld3(s->cn[c]);
            V3 t1, t2;
            s->tangents(c, &t1, &t2);
            f = n * s->rows()[3 * c].lam + t1 * s->rows()[3 * c + 1].lam + t2 * s->rows()[3 * c + 2].lam;
          }
          if (bA == b) F = F + f;
          if (bB == b) F = F - f;
        }
        ncf_out[3 * b] = F.x * ihc;
        ncf_out[3 * b + 1] = F.y * ihc;
        ncf_out[3 * b + 2] = F.z * ihc;
      }
    }
    fk<POSE>();  // post-step pose for the sensor body frames
    const float ih = prcp(h);  // impulses -> forces
    const int NS = m->num_sensors;
    if constexpr (T >= 32 && !OBJ) {
      if (sens_out && NS > 0) sensors_by_team_sums(sens_out, NS);
    } else if (sens_out && NS > 0) {
#if MG_SENSOR_MASKS
      // which sensors' bodies each contact touches, one lane per contact (chunks of T lanes), as per-sensor bit masks
      // by ballots: sensor lane j then visits only its own contacts (a foot has one or two) instead of scanning all
      // of them with two dependent LDS lookups each; same contacts, same increasing order, so the same sums bit for bit
      static_assert(MC <= 64, "the per-sensor contact masks are one 64-bit word");
      unsigned long long own = 0ull;
      const int nc = s->ncon;
      for (int c0 = 0; c0 < nc; c0 += T) {
        const int c = c0 + tl;
        int bA = -1, bB = -1;
        if (c < nc) {
          const int gA = cside(c, 2), gB = cside(c, 3);
          bA = gA >= 0 ? mt->gbody[gA] : -1;
          bB = gB >= 0 ? mt->gbody[gB] : -1;
        }
        for (int j = 0; j < NS; j++) {
          const int sb = m->sensor_body[j];
          const unsigned long long bits = (__ballot(bA == sb || bB == sb) >> tb) & team_bits<T>();
          if (tl == j) own |= bits << c0;
        }
      }
#endif
      if (tl < NS) {
      const int body = m->sensor_body[tl], nd = m->body_node[body];
      M3 Rn;
      for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) Rn.m[a][b] = s->R[nd][3 * a + b];
      M3 Rb = mul(Rn, quat_to_mat(m->body_quat[body][0], m->body_quat[body][1], m->body_quat[body][2],
                                  m->body_quat[body][3]));
      V3 xb = ld3(s->x[nd]) + mul(Rn, ld3(m->body_pos[body]));
      V3 F = v3(0, 0, 0), Tq = v3(0, 0, 0);
#if MG_SENSOR_MASKS
      for (unsigned long long mm = own; mm; mm &= mm - 1ull) {
        const int c = __builtin_ctzll(mm);
        const float sg = (cside(c, 2) >= 0 && mt->gbody[cside(c, 2)] == body) ? 1.0f : -1.0f;
#else
      for (int c = 0; c < s->ncon; c++) {
        float sg = 0.0f;
        if (cside(c, 2) >= 0 && mt->gbody[cside(c, 2)] == body) sg = 1.0f;
        else if (cside(c, 3) >= 0 && mt->gbody[cside(c, 3)] == body) sg = -1.0f;
        if (sg == 0.0f) continue;
#endif
        V3 f;
        if constexpr (L::kCompact) {
          f = ld3(s->fc(c)) * (sg * ih);
        } else {
          const V3 n = ld3(s->cn[c]), t1 = ld3(s->ct1[c]), t2 = ld3(s->ct2[c]);  // build_rows' basis
          f = (n * s->rows()[3 * c].lam + t1 * s->rows()[3 * c + 1].lam + t2 * s->rows()[3 * c + 2].lam) * (sg * ih);
        }
        F = F + f;
        Tq = Tq + cross(ld3(s->cp[c]) - xb, f);
      }
      V3 Fl = mulT(Rb, F), Tl = mulT(Rb, Tq);
      float* o = sens_out + 6 * tl;
      o[0] = Fl.x; o[1] = Fl.y; o[2] = Fl.z; o[3] = Tl.x; o[4] = Tl.y; o[5] = Tl.z;
      }
    }
    if (dforce_out && node > 0) {
      const float* np = nprop(node);
      float t = tau + ttend;
      if (np[6] > 0.0f) {
        const float fe = np[6] * (tgt - qj) - np[2] * nu;
        t += (sat & 1) ? (fe > 0.0f ? np[7] : -np[7]) : fe;
      } else {
        t += -np[2] * nu - np[3] * qj;
      }
#ifndef MG_NO_FRICTIONLOSS
      const float fl = np[8];
#else
      const float fl = 0.0f;
#endif
      if (fl > 0.0f) t -= fl * ptanh(nu * (1.0f / MG_FRICTIONLOSS_VS));  // the joint friction at the post-step state
      // the node's own limit rows of the last substep (lower, then upper: consecutive from the index build_rows
      // kept in sat), instead of a scan over every limit row
      if constexpr (L::kCompact) {
        if (sat & 2) t += llo * ih;
        if (sat & 4) t -= lhi * ih;
      } else {
        const int lr = 3 * s->ncon + (sat >> 3);
        if (sat & 2) t += s->rows()[lr].lam * ih;
        if (sat & 4) t -= s->rows()[lr + ((sat >> 1) & 1)].lam * ih;
      }
      dforce_out[node - 1] = t;
    }
  }

  // ---------------------------------------------------------------- state I/O (gym layouts)
  __device__ __forceinline__ void load(const float* root, const float* dof, const float* act_tau, const float* orow = nullptr,
                       const float* tg = nullptr) {
    // root pose/twist: every lane reads the 13 floats (one cache line pair per actor) and normalises the
    // quaternion itself (the same operations on every lane: no shuffles from the leader)
    {
      p0 = ld3(root);
      if (MG_LOAD_RSQ && freeb) {
        // free-base roots: a 1-ulp reciprocal square root instead of a correctly rounded root and four divisions
        // (~60 instructions; the fixed-base hand and Cartpole keep the exact form, their parity cases being tighter)
        const float in = prsq(root[3] * root[3] + root[4] * root[4] + root[5] * root[5] + root[6] * root[6]);
        for (int k = 0; k < 4; k++) q0[k] = root[3 + k] * in;
      } else {
        float n = sqrtf(root[3] * root[3] + root[4] * root[4] + root[5] * root[5] + root[6] * root[6]);
        for (int k = 0; k < 4; k++) q0[k] = root[3 + k] / n;
      }
    }
    if (freeb && tl < 6) {
      M3 Rr = quat_to_mat(q0[0], q0[1], q0[2], q0[3]);
      V3 cw = mul(Rr, ld3(m->body_com[0]));
      V3 om = ld3(root + 10);
      V3 vo = ld3(root + 7) - cross(om, cw);
      float tw[6] = {om.x, om.y, om.z, vo.x, vo.y, vo.z};
      nu = tw[tl];
    }
    if (node > 0) {
      qj = dof[2 * (node - 1)];
      nu = dof[2 * (node - 1) + 1];
      tau = act_tau ? act_tau[node - 1] : 0.0f;
      tgt = tg ? tg[node - 1] : 0.0f;
    }
    if (OBJ && orow) {  // object row [p, q, v_com, w]: pose on every lane, twist on the object lanes
      op = ld3(orow);
      const float n = sqrtf(orow[3] * orow[3] + orow[4] * orow[4] + orow[5] * orow[5] + orow[6] * orow[6]);
      for (int k = 0; k < 4; k++) oq[k] = orow[3 + k] / n;
      if (objl) {
        const int k = tl - ob0;
        nu = k < 3 ? orow[10 + k] : orow[7 + k - 3];
      }
    }
  }

  // writes the post-step state into the team's LDS staging (root[13], dof[2 nD])
  __device__ __forceinline__ void stage_state() {
    float w0 = __shfl(nu, tb + 0), w1 = __shfl(nu, tb + 1), w2 = __shfl(nu, tb + 2);
    float v0 = __shfl(nu, tb + 3), v1 = __shfl(nu, tb + 4), v2 = __shfl(nu, tb + 5);
    if (tl == 0) {
      s->st().root[0] = p0.x; s->st().root[1] = p0.y; s->st().root[2] = p0.z;
      for (int k = 0; k < 4; k++) s->st().root[3 + k] = q0[k];
      if (freeb) {
        M3 Rr = quat_to_mat(q0[0], q0[1], q0[2], q0[3]);
        V3 cw = mul(Rr, ld3(m->body_com[0]));
        V3 om = v3(w0, w1, w2);
        V3 vc = v3(v0, v1, v2) + cross(om, cw);
        s->st().root[7] = vc.x; s->st().root[8] = vc.y; s->st().root[9] = vc.z;
        s->st().root[10] = om.x; s->st().root[11] = om.y; s->st().root[12] = om.z;
      }
    }
    if (node > 0) {
      s->st().dof[2 * (node - 1)] = qj;
      s->st().dof[2 * (node - 1) + 1] = nu;
    }
    if (OBJ) {
      const float o0 = __shfl(nu, tb + ob0), o1 = __shfl(nu, tb + ob0 + 1), o2 = __shfl(nu, tb + ob0 + 2);
      const float o3 = __shfl(nu, tb + ob0 + 3), o4 = __shfl(nu, tb + ob0 + 4), o5 = __shfl(nu, tb + ob0 + 5);
      if (tl == 0) {
        s->oroot[0] = op.x; s->oroot[1] = op.y; s->oroot[2] = op.z;
        for (int k = 0; k < 4; k++) s->oroot[3 + k] = oq[k];
        s->oroot[7] = o3; s->oroot[8] = o4; s->oroot[9] = o5;
        s->oroot[10] = o0; s->oroot[11] = o1; s->oroot[12] = o2;
      }
    }
  }

  // gym rigid-body state of articulation body `b` (post-step FK in LDS): body-origin pose, COM linear
  // velocity, angular velocity (oracle body_states)
  __device__ __forceinline__ void body_state(int b, float* o) const {
    const int nd = m->body_node[b];
    M3 Rn;
    for (int a = 0; a < 3; a++)
      for (int c2 = 0; c2 < 3; c2++) Rn.m[a][c2] = s->R[nd][3 * a + c2];
    const M3 Rb = mul(Rn, quat_to_mat(m->body_quat[b][0], m->body_quat[b][1], m->body_quat[b][2], m->body_quat[b][3]));
    const V3 xb = ld3(s->x[nd]) + mul(Rn, ld3(m->body_pos[b]));
    const V3 r = xb + mul(Rb, ld3(m->body_com[b])) - ld3(s->x[0]);
    const V3 w = ld3(s->V[nd]), vo = ld3(s->V[nd] + 3);
    const V3 vc = vo + cross(w, r);
    float q[4];
    mat_to_quat(Rb, q);
    o[0] = xb.x; o[1] = xb.y; o[2] = xb.z;
    o[3] = q[0]; o[4] = q[1]; o[5] = q[2]; o[6] = q[3];
    o[7] = vc.x; o[8] = vc.y; o[9] = vc.z;
    o[10] = w.x; o[11] = w.y; o[12] = w.z;
  }
};

#pragma float_control(pop)

}  // namespace mg
