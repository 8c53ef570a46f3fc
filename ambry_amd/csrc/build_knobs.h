// build_knobs.h -- every compile-time A/B knob of libambrycrc with its product default, in one
// place. A knob is overridden only from the compiler command line (-DAMBRY_X=v, tools/ab_build.sh);
// ambrycrc_version() names every knob whose value differs from the default below, so a library
// that is not the product build says so (tests/test_abi.py asserts the in-tree build reports none).
//
// Probe knobs (AMBRY_*_PROBE != 0) remove work from a kernel to time what is left: those builds
// return WRONG CRCs. They compile only together with -DAMBRY_AB_PROBE_BUILD, and ambrycrc_init
// refuses to start such a library unless AMBRYCRC_ALLOW_PROBE=1 is in the environment.
#pragma once

// ---- message verify / transform (message_kernels.hip)
#ifndef AMBRY_PROPS_WIN  // bytes of a record staged per thread in LDS for the properties parse
#define AMBRY_PROPS_WIN 96
#endif
#ifndef AMBRY_PARSE_BPC  // parse-kernel blocks per CU (0: one thread per message)
#define AMBRY_PARSE_BPC 2
#endif
#ifndef AMBRY_REGION_WPE  // region pass 2: waves per SIMD the register budget allows
#define AMBRY_REGION_WPE 2
#endif
#ifndef AMBRY_REGION_BPC_SMALL  // the same for regions of <= 1.5 KiB per message
#define AMBRY_REGION_BPC_SMALL 2
#endif
#ifndef AMBRY_REGION_BPC  // region pass 2: blocks per CU (0: one thread per message)
#define AMBRY_REGION_BPC 2
#endif
#ifndef AMBRY_REGION_AUX  // region pass 2's LDS helpers (region_crc.h Aux): 1 = LDS byte masks + H0, 2 = x^(8*256)
#define AMBRY_REGION_AUX 7  // byte tables for the Horner steps, 4 = two-multiply un-shift
#endif
#ifndef AMBRY_STREAM_PIPE  // serialize copy mode's streamed form: message i+1's loads in flight while i is hashed
#define AMBRY_STREAM_PIPE 1
#endif
#ifndef AMBRY_SEAL_BPC  // serialize copy mode's streamed form: put_stream_seal_kernel blocks per CU
#define AMBRY_SEAL_BPC 2
#endif
#ifndef AMBRY_HOST_VERIFY_CPU_PCT  // host verify's CPU leg before it is measured: this % of the CRC rate
#define AMBRY_HOST_VERIFY_CPU_PCT 50
#endif
#ifndef AMBRY_HOST_XFORM_CPU_PCT  // the same for the host transform's CPU leg
#define AMBRY_HOST_XFORM_CPU_PCT 25
#endif
#ifndef AMBRY_FUSED_PROC  // one-pass region verify: processor waves per workgroup (0: per call)
#define AMBRY_FUSED_PROC 0
#endif
#ifndef AMBRY_FUSED_WAVES_VERIFY  // one-pass region kernel, verify form: waves per workgroup (one per CU)
#define AMBRY_FUSED_WAVES_VERIFY 12
#endif
#ifndef AMBRY_FUSED_WAVES_COPY  // the same, the transform's copy form
#define AMBRY_FUSED_WAVES_COPY 8
#endif
#ifndef AMBRY_FUSED_NT  // one-pass region kernel: nontemporal streamer loads (0: temporal, the lines stay in L2)
#define AMBRY_FUSED_NT 1
#endif
#ifndef AMBRY_FUSED_ENDS  // one-pass processors hash a record's head / tail runs right after the parse, before
#define AMBRY_FUSED_ENDS 1  // the wait for its run sums: 0 = never, 1 = the transform's copy form, 2 = also the verify
#endif

// ---- batch CRC kernels (crc32_kernels.hip, crc32_kernels.h, ambrycrc_ctx.h)
#ifndef AMBRY_GRP_PRIO  // s_setprio 3 around the streamed group path's loads
#define AMBRY_GRP_PRIO 0
#endif
#ifndef AMBRY_GRP_IL  // chunks interleaved per group round of the group phase
#define AMBRY_GRP_IL 4
#endif
#ifndef AMBRY_C0_G  // lanes per chunk of size class 0
#define AMBRY_C0_G 2
#endif
#ifndef AMBRY_C0_NB  // class-0 chunks per wave round
#define AMBRY_C0_NB 8
#endif
#ifndef AMBRY_C1_MAX  // the largest class-1 (8-lane group) chunk
#define AMBRY_C1_MAX 1024
#endif
#ifndef AMBRY_RUNS_STORE_NT  // region pass 1: nontemporal run-sum stores
#define AMBRY_RUNS_STORE_NT 0
#endif
#ifndef AMBRY_RUNS_NT  // region pass 1: nontemporal loads (0: temporal -- pass 2's re-reads may then hit L2 / MALL)
#define AMBRY_RUNS_NT 1
#endif
#ifndef AMBRY_RUNS_GIL  // region pass 1: super-blocks in flight per wave beyond the current one
#define AMBRY_RUNS_GIL 1
#endif
#ifndef AMBRY_PLAN_PER_BLOCK  // chunks per plan-kernel block
#define AMBRY_PLAN_PER_BLOCK 2048
#endif
#ifndef AMBRY_DEFAULT_VARIANT  // kernel variant a context starts with (kVariantDefault)
#define AMBRY_DEFAULT_VARIANT 29
#endif

// ---- probes (timing only, wrong CRCs)
#ifndef AMBRY_REGION_PROBE  // 1 = records not CRC'd, 2 = no run-sum loads, 3 = no head / tail loads
#define AMBRY_REGION_PROBE 0
#endif
#ifndef AMBRY_RUNS_PROBE  // 1 = no run sums into LDS, 5 = no global stores, 6 = stores to one line set
#define AMBRY_RUNS_PROBE 0
#endif
// (The one-pass kernel's timing probes, round 5's AMBRY_FUSED_PROBE 1-5, live in
// tools/probes/fused_probe_branches.patch: `git apply` it to a scratch tree to rebuild them.)

#if (AMBRY_REGION_PROBE != 0 || AMBRY_RUNS_PROBE != 0 || defined(AMBRYCRC_DIAGNOSTICS) || \
     defined(AMBRY_AB_SPLIT_GROUP)) && !defined(AMBRY_AB_PROBE_BUILD)
#error "probe / diagnostic knobs build a library that returns wrong CRCs or runs unshipped kernels: define AMBRY_AB_PROBE_BUILD (tools/ab_build.sh does)"
#endif

// X(name, default) for every knob above: ambrycrc_version() reports those that differ.
#define AMBRY_KNOB_LIST(X)                                                                                  \
  X(AMBRY_PROPS_WIN, 96) X(AMBRY_PARSE_BPC, 2) X(AMBRY_REGION_WPE, 2) X(AMBRY_REGION_BPC, 2)                  \
  X(AMBRY_REGION_BPC_SMALL, 2) X(AMBRY_REGION_AUX, 7) X(AMBRY_SEAL_BPC, 2) X(AMBRY_STREAM_PIPE, 1) X(AMBRY_HOST_VERIFY_CPU_PCT, 50) X(AMBRY_HOST_XFORM_CPU_PCT, 25)                                                                          \
  X(AMBRY_FUSED_PROC, 0)                                                                                      \
  X(AMBRY_FUSED_WAVES_VERIFY, 12)                                                                               \
  X(AMBRY_FUSED_WAVES_COPY, 8) X(AMBRY_FUSED_NT, 1) X(AMBRY_FUSED_ENDS, 1)                                                                 \
  X(AMBRY_GRP_PRIO, 0) X(AMBRY_GRP_IL, 4) X(AMBRY_C0_G, 2) X(AMBRY_C0_NB, 8) X(AMBRY_C1_MAX, 1024)           \
  X(AMBRY_RUNS_STORE_NT, 0) X(AMBRY_RUNS_NT, 1) X(AMBRY_RUNS_GIL, 1) X(AMBRY_PLAN_PER_BLOCK, 2048) X(AMBRY_DEFAULT_VARIANT, 29) \
  X(AMBRY_REGION_PROBE, 0) X(AMBRY_RUNS_PROBE, 0)

#if defined(AMBRY_AB_PROBE_BUILD)
#define AMBRY_IS_PROBE_BUILD 1
#else
#define AMBRY_IS_PROBE_BUILD 0
#endif
