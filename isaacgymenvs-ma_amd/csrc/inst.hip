// inst.hip — one capacity instance of the team kernels per translation unit (build.py compiles this
// file once per -DMG_INST=i, i < MG_NUM_INST, in parallel, and links the objects with migym.hip).
#include "step_kernels.hpp"

#ifndef MG_INST
#error "compile with -DMG_INST=<instance index> (build.py)"
#endif
static_assert(MG_INST >= 0 && MG_INST < MG_NUM_INST, "MG_INST out of range");

namespace mgi {
constexpr InstDesc kI = kInst[MG_INST];
template struct BuildTile<kI.T, kI.MN, kI.MC, kI.MG, kI.MP, kI.OBJ, kI.LAY>;
template struct RunSimulate<kI.T, kI.MN, kI.MC, kI.MG, kI.MP, kI.OBJ, kI.LAY>;
template struct RunEnvStep<kI.T, kI.MN, kI.MC, kI.MG, kI.MP, kI.OBJ, kI.LAY>;
template int phase_buf_publish<MG_INST>(unsigned long long*);
}  // namespace mgi
