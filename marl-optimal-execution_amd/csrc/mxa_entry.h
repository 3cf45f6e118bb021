// mxa_entry.h — the kernels of one configuration as seen by the C-ABI (mxa_api.hip).
//
// Each configuration's engine is compiled in a translation unit of its own (mxa_inst.hip built
// with -DMXA_INST_CFG=<id>), so the eight engine instantiations build in parallel; the C-ABI
// picks a configuration's launchers through mxa_entry_<id>().
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/mxa.h"
#include "mxa_layout.h"

typedef void (*mxa_build_fn)(dim3, dim3, size_t, hipStream_t, char*, uint64_t, int, const uint32_t*, const uint8_t*,
                             const RpCtx*);
typedef void (*mxa_run_fn)(dim3, dim3, size_t, hipStream_t, char*, uint64_t, int, int, int64_t, const RpCtx*, BlRec*,
                           int, const int32_t*);
typedef void (*mxa_stop_fn)(dim3, dim3, size_t, hipStream_t, char*, uint64_t, int, mxa_agent_final*, BlRec*, int,
                            const RpCtx*);
typedef void (*mxa_step_fn)(dim3, dim3, size_t, hipStream_t, char*, uint64_t, int, int, int64_t, const RpCtx*,
                            const double*, double*, int32_t*);

typedef void (*mxa_step_many_fn)(dim3, dim3, size_t, hipStream_t, char*, uint64_t, int, int, int64_t, const RpCtx*,
                                 const double*, double*, int32_t*, int);

typedef int (*mxa_occ_fn)(size_t);  // resident blocks (envs) per CU of the measured kernel at that LDS size

struct MxaEntry {
  mxa_build_fn build;
  mxa_run_fn run, run_log;     // run_log: the book-update-log variant (plain Kernel.runner configs)
  mxa_run_fn run_fast;         // without the parity instrumentation (hash off, no trace ring)
  mxa_stop_fn stop, stop_log;
  mxa_step_fn step, step_fast; // GymKernel configurations (step_fast: without the instrumentation)
  mxa_step_many_fn step_many, step_many_fast;  // k steps per launch, actions given up front
  mxa_occ_fn occ;              // hipOccupancyMaxActiveBlocksPerMultiprocessor of run_fast / step_fast
};

MxaEntry mxa_entry_0();
MxaEntry mxa_entry_1();
MxaEntry mxa_entry_2();
MxaEntry mxa_entry_3();
MxaEntry mxa_entry_4();
MxaEntry mxa_entry_5();
MxaEntry mxa_entry_6();
MxaEntry mxa_entry_7();
MxaEntry mxa_entry_8();
MxaEntry mxa_entry_9();
MxaEntry mxa_entry_10();
MxaEntry mxa_entry_11();
MxaEntry mxa_entry_12();
MxaEntry mxa_entry_13();
MxaEntry mxa_entry_14();
MxaEntry mxa_entry_15();
MxaEntry mxa_entry_16();
MxaEntry mxa_entry_17();
#define MXA_N_CONFIGS 18
