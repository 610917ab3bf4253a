// common.hpp — host-side pieces shared by the C-ABI translation unit (migym.hip) and the
// per-instance kernel translation units (inst.hip): the sim handle and the error channel.
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/migym.h"

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
  // work ordering of the fused step (32-lane instances: K = 1 from 16,384 envs, 8 below; else off;
  // MIGYM_ORDER_EVERY = K overrides at mg_sim_create): every K-th mg_env_step
  // first sorts the envs by their last step's constraint-row count, descending (k_order), and the step kernels
  // take their envs in that order -- teams of similar cost share a wave (the wave runs its slowest team's rows)
  // and the heavy envs start first.  Envs are independent, so every result is the same bit for bit.
  int order_every;
  long long order_steps;
  bool order_valid;
  int* d_order;        // (n / A) env slots -> env
  unsigned char* d_cost; // (n) the last step's row count per actor (saturated at 255)
  // kernel spans (mg_kernel_span_begin): per recorded launch, span_stride (start, end) pairs, one per wave
  unsigned long long* d_span;
  int span_cap, span_next, span_stride;
  int span_waves[1024];  // waves of each recorded launch
};

// the step kernels' ordering arguments (nullptr order: slot = env)
struct MgOrder {
  const int* order;
  unsigned char* cost;
  unsigned long long* clk;  // nullptr, or this launch's span slot (mg_kernel_span_begin)
};

namespace mgi {
constexpr int kBlock = 64;
// sets mg_last_error() (thread-local, defined in migym.hip) and returns `code`
int fail(int code, const std::string& msg);
}  // namespace mgi
