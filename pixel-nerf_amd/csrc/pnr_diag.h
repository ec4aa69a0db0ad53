// Diagnostic builds of the ray-march kernels: every build knob the kernels still read.
//
// None of these is defined in the shipped build (pixel-nerf_amd/Makefile); a diagnostic library
// is built next to it with scripts/build_variant.sh NAME WORKTREE -D<knob> and loaded through
// PNR_LIB_PATH by the probes under tools/.  The knobs never change the kernels' schedule in the
// default build: each one either adds timers (timing builds, valid results) or removes a piece of
// work (ablation builds, results INVALID, used only to bound what that piece costs).
//
// Timing (valid results):
//   PNR_PHASE_TIMING   k_point_mlp: shader cycles per phase of the recorded wave (PT / PT_COUNT
//                      stamps, slots below), summed over workgroups; read by pnr_debug_phase
//                      (tools/mlp_probe.py).  PNR_PT_WAVE=w records wave w (default 0).
//   PNR_EPI_TIMING     the fused march epilogue (march_ray / sample_fine_wave): cycles of its
//                      composite, cdf, draws and sort; read by pnr_debug_epi (tools/gpu_epi_probe.sh).
//   PNR_WGH_STATS      k_wgrad_h: scale-move statistics (pnr_wgrad_stats, tools/wgrad_stats.py).
//
// Ablations (results invalid; tools/probe_ablate.sh, tools/wstream_ab.sh):
//   PNR_GEMM_ONLY        k_point_mlp runs only its GEMM chain on constant operands (no features,
//                        gather, publishes or head).
//   PNR_ABLATE_WSTREAM   every k-step re-reads k-step 0's weight fragments (no L2 weight stream).
//   PNR_ABLATE_GATHER    no projected-latent / latent row loads (the gather records stand in).
//   PNR_ABLATE_PUBSTORE  the relu publish's image stores are removed.
//   PNR_ABLATE_PUBSPLIT  the relu publish stores the raw value bits: no relu, scale, fp16 split or
//                        permlane exchange (the stores and the column maxima stay).
//   PNR_ABLATE_CMAXREAD  the relu publish takes constant column exponents: no column-maximum reads.
//   PNR_ABLATE_BIAS      constants instead of bias loads.
//   PNR_ABLATE_SAVEF     the training forward's fp32 activation-save stores (the relu slots) removed.
//   PNR_ABLATE_SAVEM     the training forward's relu sign-mask stores removed.
//   PNR_ABLATE_SPLIT     split-bf16 modes: the hi part only, no split VALU.
//   PNR_ABLATE_STGREAD   split-bf16 modes: B operands from registers instead of the staging ring.
//   PNR_ABLATE_KBARRIER  split-bf16 modes: no barrier between k-steps.
//   PNR_WG_NOPUT, PNR_WG_MFMA3, PNR_WG_L2ROWS, PNR_WGH_HEAD, PNR_WGH_INIT
//                        wgrad.hip: stale images, 3 of 6 products, L2-hot rows, and the
//                        k_wgrad_h split pieces (tools/wgrad_probe.py).
//
// Rejected schedule variants are not knobs: each is a patch under tools/patches/ with its
// same-box A/B result in the header, applied to a work tree by scripts/build_variant.sh.
#pragma once
#include <cstdint>

// Included by mlp.hip only (it defines the counters; march_dev.h's epilogue stamps are no-ops in
// every other translation unit).
#ifdef PNR_EPI_TIMING
__device__ unsigned long long g_epi[8];
#define EPI_DECL uint64_t epi_last_ = __builtin_amdgcn_s_memtime();
#define EPI_T(i)                                                                  \
    do {                                                                          \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();                         \
        if (lane == 0) atomicAdd(&g_epi[i], (unsigned long long)(t_ - epi_last_)); \
        epi_last_ = t_;                                                           \
    } while (0)
#else
#define EPI_DECL
#define EPI_T(i) ((void)0)
#endif

// k_point_mlp phase slots (wave cycles per tile, summed): 0 features + projection, 1 latent
// gather / projected-row stage, 2 GEMMs, 3 glue (bias, barriers), 4 lin_out head, 5 GEMM calls,
// 6 tiles, 8-12 feature sub-phases, 13 colmax VALU, 14 colmax barrier, 15 split + stores,
// 16 barrier after the stores, 17 ring prime + bias loads before a publish.
#ifdef PNR_PHASE_TIMING
#define PT(gc, i)                                                     \
    do {                                                              \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();             \
        (gc).pt[i] += t_ - (gc).pt_last;                              \
        (gc).pt_last = t_;                                            \
    } while (0)
#define PT_COUNT(gc, i) ((gc).pt[i] += 1)
#define PT_WAIT() asm volatile("s_waitcnt vmcnt(0)" ::: "memory")
#ifndef PNR_PT_WAVE
#define PNR_PT_WAVE 0
#endif
#else
#define PT_WAIT() ((void)0)
#define PT(gc, i) ((void)0)
#define PT_COUNT(gc, i) ((void)0)
#endif
