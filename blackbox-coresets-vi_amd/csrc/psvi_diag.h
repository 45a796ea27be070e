/* psvi_diag.h -- diagnostics of libpsvi_hip.so: ablation masks, A/B switches
   between a kernel and its fallback, per-workgroup phase stamps.  Internal to
   the library and its profiling tools (tools/, some A/B tests); never needed
   for results, and not part of the drop-in interface (include/psvi_hip.h).
   Every key costs nothing while unset. */
#ifndef PSVI_DIAG_H
#define PSVI_DIAG_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PSVI_DBG_NET_ABLATION 1  /* value: mask of network-kernel parts to skip
                                    (1 loads, 2 fwd GEMMs, 4 loss head, 8
                                    backward, 16 global dW writes); 0 = full   */
int psvi_debug_set(int32_t key, int32_t value);
#define PSVI_DBG_NET_STAMPS 2    /* ptr: device uint64 buffer, 16 slots per
                                    network-kernel workgroup: s_memtime at
                                    phase boundaries (1 loads, 9..11 forward
                                    layers, 2 forward, 3 head, 4..8 backward
                                    phases, 12 end; 13 / 14 s_memrealtime
                                    start / end)                               */
#define PSVI_DBG_UPD_ABLATION 3  /* value: mask of full-cov update-kernel parts to
                                    replace (1 G/eps loads by one cached
                                    address, 2 dL MFMAs skipped, 4 corr/m/v
                                    loads by one address, 8 stores skipped,
                                    16 fused-sample MFMAs skipped, 32 eps_next
                                    loads by one address, 64 Adam math by an
                                    add)                                       */
#define PSVI_DBG_UPD_STAMPS 4    /* ptr: device uint64 buffer, 16 slots per
                                    update-kernel workgroup (start, staged,
                                    loop done, end, HW_ID, XCC_ID; S <= 128:
                                    6..11 = summed shader clocks of eps stage
                                    1, MFMA half 1, stage 2, MFMA half 2,
                                    epilogue, fused-sample GEMM)               */
#define PSVI_DBG_NET_SPLIT_BELOW 5 /* value: give each sample two network
                                    workgroups (gradient roles; pseudopoint
                                    chunks if still short of CUs) when a rank has
                                    fewer samples than this (plans created
                                    afterwards; default 256)                   */
#define PSVI_DBG_FWD_ABLATION 6  /* value: mask of full-cov sample-kernel parts to
                                    skip (1 loads, 2 MFMAs, 4 x atomics)       */
#define PSVI_DBG_FWD_STAMPS 7    /* ptr: device uint64 buffer, 16 slots per
                                    sample-kernel workgroup (start, first stage,
                                    MFMAs done, end, HW_ID, XCC_ID)            */
int psvi_debug_set_ptr(int32_t key, void* ptr);
#define PSVI_DBG_LOOP_TIMING 8   /* value: record HIP events around the network and
                                    the update launches of every value-th step of
                                    full-cov psvi_inner_loop calls (0 = off;
                                    setting it drops earlier records)          */
#define PSVI_DBG_UPD_CHUNK 9     /* value: c-blocks (64x64 tiles) per full-cov update
                                    chunk for plans created afterwards (0 = auto:
                                    about one chunk per resident workgroup)    */
#define PSVI_DBG_UPD_STREAM_OFF 10 /* value: 1 = the tiled fused update runs the
                                    chunked kernel instead of the streaming one
                                    (A/B diagnostics; 0 = streaming)           */
#define PSVI_DBG_STREAM_WGS 11   /* value: workgroups of the streaming update for
                                    plans created afterwards (0 = 256)         */
#define PSVI_DBG_STREAM_RR 12    /* value: 1 = the streaming update's runs dealt
                                    round-robin over the XCDs instead of one
                                    contiguous eighth per XCD (plans created
                                    afterwards; A/B diagnostics)               */
#define PSVI_DBG_NET_THREADS 14  /* value: threads per network workgroup (256 or
                                    512; 0 = by chunk size) for plans created
                                    afterwards (A/B diagnostics)               */
#define PSVI_DBG_NET_WG_TARGET 15 /* value: network workgroups a split rank aims
                                    for (pseudopoint chunks added until samples x
                                    roles x chunks reach it; default 256) for
                                    plans created afterwards (A/B diagnostics) */
#define PSVI_DBG_LENET_ABLATION 17 /* value: mask of LeNet MFMA-backward parts to
                                    skip (timing diagnostics; wrong results):
                                    1 d P1 GEMM, 2 dW2, 4 patch sums, 8 dW1,
                                    16 image load, 32 P1 load                  */
#define PSVI_DBG_ROP_STAMPS 18   /* ptr: device uint64 buffer, 16 slots per
                                    R-op workgroup (sample + split * S): shader
                                    clocks summed per phase (tools/rop_stamps.py) */
#define PSVI_DBG_KSTREAM_OFF 19  /* value: 1 = the chunked update kernel instead of
                                    the K-split streaming one at S > 128 (A/B) */
#define PSVI_DBG_NET_SCALAR_LOADS 20 /* value: 1 = the full-cov network kernel's
                                    scalar x / u load path instead of the float4
                                    one (A/B)                                   */
#define PSVI_DBG_KSTREAM_WGS 21      /* value: workgroups of the K-split update
                                    for plans created afterwards (0: 512)       */
#define PSVI_DBG_FWD_SEG_OFF 22      /* value: 1 = the item-grid sample kernel instead
                                    of the segmented one at S > 128 (A/B)       */
#define PSVI_DBG_NET_MLOOP_OFF 23     /* value: 1 = a full-cov plan whose pseudopoints
                                    exceed the network kernel's LDS runs one
                                    workgroup per chunk with per-chunk slots
                                    and a slot sum, instead of looping the
                                    chunks inside each workgroup (A/B)          */
#define PSVI_DBG_STREAM_BF_OFF 24     /* value: 1 = the tiled inner loop's streaming
                                    update on the fp32 matrix instructions
                                    instead of the bf16-piece (fp32-faithful)
                                    kernel (A/B)                               */
#define PSVI_DBG_BF_STAMPS 25        /* ptr: device uint64 buffer, 16 slots per
                                    workgroup of the bf16-piece streaming
                                    update: shader clocks summed per phase
                                    (tools/bf_stamps.py)                       */
#define PSVI_DBG_FWD_SEG_BF_OFF 26   /* value: 1 = the segmented sample (K = S > 128)
                                    on the fp32 MFMA kernel instead of the
                                    bf16-piece (fp32-faithful) one (A/B)      */
#define PSVI_DBG_KSTREAM_BF_OFF 27   /* value: 1 = the K-split update (K = S > 128)
                                    on the fp32 MFMA kernel instead of the
                                    bf16-piece (fp32-faithful) one (A/B)      */
#define PSVI_DBG_ROP_VALU 29         /* value: 1 = the R-op (psvi_hvp's tangent
                                    forward and R-backward) on the VALU kernel
                                    (the form for row blocks past the LDS)
                                    instead of the matrix-core one (A/B)       */
#define PSVI_DBG_FWD_PAIR_BF 31      /* value: 0 = psvi_hvp's sample pair (x and its
                                    tangent) on the fp32 item grid instead of
                                    the paired bf16-piece segmented launch
                                    (default 1; A/B)            */
#define PSVI_DBG_NET_GEO_OFF 30      /* value: 1 = the network kernel's run-time
                                    geometry for the fn2 64-40-40-2 stack too,
                                    instead of its compile-time one (A/B)      */
#define PSVI_DBG_STREAM_COST 34      /* value: first-tile% + 1000 x diagonal-tile%:
                                    the streaming update's extra cost weights of
                                    a band's first and diagonal (last) tiles in
                                    the run partition (-1: the defaults; set
                                    before creating the plan; tuning)          */
#define PSVI_DBG_STREAM_FOLD_OFF 32  /* value: 1 = the streaming update's band
                                    combine (x' = mean + softplus(sd) eps' + the
                                    band's slots) as mvn_fwd_reduce_kernel
                                    instead of in the kernel (A/B)             */
/* mean device microseconds of the recorded windows: out[0] network kernel,
   out[1] update (+ its slot reduce), out[2] windows; synchronizes on them and
   drops the records */
int psvi_debug_loop_timing(double* out);


#ifdef __cplusplus
}
#endif
#endif /* PSVI_DIAG_H */
