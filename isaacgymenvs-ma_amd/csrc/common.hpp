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
};

namespace mgi {
constexpr int kBlock = 64;
// sets mg_last_error() (thread-local, defined in migym.hip) and returns `code`
int fail(int code, const std::string& msg);
}  // namespace mgi
