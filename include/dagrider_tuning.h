/*
 * dagrider_tuning.h -- kernel-tuning hook of the PROFILING build only
 * (dag_rider_amd/libdagrider_gpu_timing.so, compiled with -DDR_TUNING).
 * The shipped library (libdagrider_gpu.so) does not export it, and the
 * tuning variants it selects are not compiled into the shipped library.
 * Used by tools/tune.py; no reference counterpart.
 */
#ifndef DAGRIDER_TUNING_H
#define DAGRIDER_TUNING_H
#include "dagrider_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Average device time of `iters` launches of one kernel variant on the
 * resident DAG.  kernel 0 = round-summary + commit pass (variant 0 shipped,
 * others alternative geometries), 1 = streaming read of the strong rows
 * (variant 0 grid-stride, 2 blocked), 2 = the replay's whole summary phase. */
int dr_profile_kernel(dr_ctx *ctx, int kernel, int variant, int iters, float *avg_ms);

#ifdef __cplusplus
}
#endif
#endif
