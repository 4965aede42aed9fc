// sit_steps_f32.hip — the float32 step kernels (k_env_steps<float, ...>) in a translation unit of
// their own, so that their device code alone is compiled with -ffast-math (reassociation,
// approximate transcendentals, finite-math).  The float64 path, every other kernel and all host
// code (derived constants, map index) stay strict in sit_kernels.hip.  The float32 contract is
// unchanged: 1e-5 relative against the oracle (tests/test_gpu_parity.py) — see DESIGN.md §4.5.

#include "sit_impl.h"

int sit_launch_steps_f32(sit_handle* h, const void* io, void* stream) {
  return launch_steps<float>(h, *static_cast<const StepIO<float>*>(io), (hipStream_t)stream);
}

// the float32 map predicates of the step kernels (sit_probe_map on a float32 handle): same TU and
// flags as the step kernels, so the probes check the code the benchmark runs
int sit_launch_probe_f32(sit_handle* h, int n, const void* pts_ne, void* dist, uint8_t* inside, uint8_t* hull,
                         void* stream) {
  return launch_probe<float>(h, n, pts_ne, dist, inside, hull, (hipStream_t)stream);
}

// the IEEE float64 helpers as compiled under this TU's fast-math flags (sit_selftest_f64)
int sit_launch_selftest_f32tu(int op, int n, const double* a, const double* b, double* out, void* stream) {
  return launch_selftest(op, n, a, b, out, (hipStream_t)stream);
}

#if defined(SIT_DIAG_PATHS) || defined(SIT_DIAG_PHASES) || defined(SIT_DIAG_SYNC) || defined(SIT_DIAG_SERVE) || defined(SIT_DIAG_PLACE)
// diagnostic builds only: this TU's counters (the float32 step kernels')
extern "C" int sit_diag_read_f32(unsigned long long* out, int reset) { return diag_read_impl(out, reset); }
#endif
#ifdef SIT_DIAG_PLACE
extern "C" int sit_diag_read_waves_f32(unsigned long long* out, int n) { return diag_read_waves_impl(out, n); }
#endif

// the float32 step kernels' blocks whose waves shared a SIMD (sit_role_fallbacks)
int sit_role_fallbacks_f32tu(unsigned long long* out, int reset) { return role_fallbacks_impl(out, reset); }

#ifdef SIT_DEBUG
// the float32 step kernels' failed bounds checks (sit_debug_flags)
int sit_debug_flags_f32tu(uint32_t* out) { return debug_flags_impl(out); }
#endif
