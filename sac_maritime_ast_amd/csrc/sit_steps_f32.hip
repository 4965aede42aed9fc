// sit_steps_f32.hip — the float32 step kernels (k_env_steps<float, ...>) in a translation unit of
// their own, so that their device code alone is compiled with -ffast-math (reassociation,
// approximate transcendentals, finite-math).  The float64 path, every other kernel and all host
// code (derived constants, map index) stay strict in sit_kernels.hip.  The float32 contract is
// unchanged: 1e-5 relative against the oracle (tests/test_gpu_parity.py) — see DESIGN.md §4.5.

#include "sit_impl.h"

int sit_launch_steps_f32(sit_handle* h, const void* io, void* stream) {
  return launch_steps<float>(h, *static_cast<const StepIO<float>*>(io), (hipStream_t)stream);
}
