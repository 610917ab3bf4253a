// common.hpp — host-side pieces shared by the C-ABI translation unit (migym.hip) and the
// per-instance kernel translation units (inst.hip): the sim handle and the error channel.
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/migym.h"

// the compact team layout (team_physics.hpp TeamLDSC): the 16- and 32-lane locomotion instances, whose
// LDS then holds twelve waves per CU.  Its ABA slots are per tree level (kCompactLevelSlots nodes at one depth at most),
// which the dispatcher checks against the model (dispatch.hpp MG_FITS)
#ifndef MG_COMPACT_LDS
#define MG_COMPACT_LDS 1
#endif
constexpr int kCompactLevelSlots = 8;
constexpr bool mg_compact_layout(int T, int MN, int OBJ) {
  return MG_COMPACT_LDS && (T == 16 || T == 32) && OBJ == 0 && MN <= 32;
}

struct mg_sim {
  mg_model host_model;
  mg_model* d_model;
  void* d_tile;     // the launched instance's model tile image (mgi::BuildTile), nullptr if none fits
  unsigned* d_wq;   // the step kernels' work-queue counters [dequeues, finished waves] (step_kernels.hpp)
  mg_sim_params params;
  int32_t n;        // actors
  int32_t device;
  mg_state_views views;
  bool bound;
  // work ordering of the fused step (step_kernels.hpp MgOrder; mg_sim_create picks the mode per instance and env
  // count, MIGYM_ORDER = off | lists | sort overrides): every mg_env_step takes its envs in descending order of
  // their constraint-row counts of the previous step -- teams of similar cost share a wave (the wave runs its slowest
  // team's rows) and the heavy envs start first.  Envs are independent, so every result is the same bit for bit.
  //   lists (kOrderLists): the previous launch built the order itself: each env appended its index to the bucket of
  //     its row count (two sets of kOrderBuckets lists, alternating launch by launch), and that launch's last wave
  //     cleared the set it had read;
  //   sort (kOrderSort): the previous launch wrote each env's row count, and a two-pass counting sort
  //     (k_ohist, k_oscatter) before the launch turns them into the permutation it reads.
  int order_mode;      // kOrderOff / kOrderLists / kOrderSort
  int lds_pad;         // dynamic LDS added to every step-kernel launch (MIGYM_LDS_PAD; occupancy experiments, 0)
  long layout_n;       // the batch the step kernels' LDS layout is picked for (MIGYM_LAYOUT; dispatch.hpp layout_fits)
  long long order_steps;  // ordered launches so far (the parity of the set the lists' launches write)
  int sort_every;      // sort: every K-th ordered launch sorts (the launches between keep the last permutation)
  bool order_valid;    // the previous ordered launch left an order for this one
  unsigned* d_bq;      // lists: [2][kOrderBuckets] bucket counts, then the launch's finished-wave counter
  int* d_blist;        // lists: [2][kOrderBuckets][bq_cap] env indices per bucket
  int bq_cap;          // env units (n / order_unit)
  int order_unit;      // actors per unit of the work order: an env's A agents (MG_SORT_WAVE_UNITS: a wave's teams)
  int order_agents;    // the agents per env the order was sized for
  int* d_order;        // sort: (bq_cap) slot -> env unit
  unsigned char* d_cost;  // sort: (bq_cap) the last launch's row count per env unit (its agents' largest, <= 255)
  unsigned* d_osort;   // sort: [kSortRep][256] bin totals, [blocks][256] the blocks' bases, then ushort ranks
  // kernel spans (mg_kernel_span_begin): per recorded launch, span_stride (start, end) pairs, one per wave
  unsigned long long* d_span;
  int span_cap, span_next, span_stride;
  int span_waves[1024];  // waves of each recorded launch
};

// the step kernels' ordering arguments: the bucket lists this launch reads (rcnt nullptr: slot = env) and writes
// (wcnt nullptr: no ordering), the read set's counts the last wave clears, the finished-wave counter
constexpr int kOrderBuckets = 32;  // row-count classes of width kOrderWidth, descending (bucket 0: 62 rows and more)
constexpr int kOrderWidth = 2;
constexpr int kOrderOff = 0, kOrderLists = 1, kOrderSort = 2;
#ifndef MG_SORT_REP
#define MG_SORT_REP 8
#endif
// sort: copies of the bin totals (block b adds into copy b % kSortRep): the hot bins' device-scope atomics spread
// over 8 words each (k_ohist 6.4 -> 4.8 us at 65,536 envs under the profiler; Ant 65,536 +0.3 %)
constexpr int kSortRep = MG_SORT_REP;
constexpr int kSortTot = kSortRep * 256;  // sort: the bin totals (zero before every sort: the step kernel that consumes
                                         // a sort's permutation clears them, MgOrder::tot_clear)
struct MgOrder {
  const int* order;     // sort: this launch's permutation (nullptr: none yet)
  unsigned char* cost;  // sort: the row counts this launch writes
  const unsigned* rcnt;
  const int* rlist;
  unsigned* wcnt;
  int* wlist;
  unsigned* rclear;  // the read set's counts (cleared by the last wave)
  unsigned* done;
  int cap;
  unsigned long long* clk;  // nullptr, or this launch's span slot (mg_kernel_span_begin)
  unsigned* tot_clear;      // sort: the bin totals, zeroed by block 0 of the step kernel (k_oscatter, their last reader,
                            // has finished: stream order), so the next sort starts from zero with no host-side state
  int unit;                 // sort: actors per unit (consecutive actors, one permutation entry; divides a wave's teams)
};
// sort units of one wave's consecutive envs (64 / T single-agent envs per unit, keyed by their largest row count):
// every wave steps 64 / T consecutive envs, so the small per-env arrays keep their lines whole (VERDICT r5 item 3's
// line-coherent units); 0: one env per unit (an MA env's agents together)
#ifndef MG_SORT_WAVE_UNITS
#define MG_SORT_WAVE_UNITS 0
#endif

namespace mgi {
constexpr int kBlock = 64;
// sets mg_last_error() (thread-local, defined in migym.hip) and returns `code`
int fail(int code, const std::string& msg);
}  // namespace mgi
