/*
 * awq_diag.h — diagnostics / A-B measurement controls, compiled ONLY into the diagnostics
 * build libawq_hip_diag.so (`make -C awq-converter_amd/csrc diag`, -DAWQ_DIAG), which
 * scripts/ and the variant tests load explicitly.  The shipped libawq_hip.so has one path
 * per shape: no awq_set_tuning symbol, none of the A/B kernel variants, the measured
 * defaults below compiled in.
 *
 * Every setting gives the same bits as the default (the GPU tests check that); only speed
 * differs.  Thread-local: it applies to launches made from the calling thread.
 */
#ifndef AWQ_DIAG_H
#define AWQ_DIAG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct awq_tuning {
    int32_t max_blocks;      /* > 0: cap the streaming kernel's grid (waves then walk many tiles) */
    int32_t tiles_per_wave;  /* > 1: tiles per wave of the streaming kernel's non-persistent grid */
    int32_t no_rowgroup;     /* 1: shapes of the row-segment kernel take the generic kernel */
    int32_t rg_waves;        /* 1 or 2: waves per row-segment tile (0 = cost model) */
    int32_t rg_gpt;          /* 8..64, multiple of 8: groups per row-segment tile (0 = cost model) */
    int32_t gen_noreg;       /* fp64 RTN: 0 the LDS span (any gs whose span fits 16 KiB), 1 the
                                strided span, 2 the register span at gs 64 / 128 (A/B) */
    int32_t dq_words_v1;     /* packed dequantize kernel: 0 the default, 1 the round-2 word kernel
                                (per-thread stores), 2 / 3 LDS-staged words with / without
                                XCD-contiguous blocks, 4 / 5 four-output lanes without / with,
                                6 / 7 batched four-output lanes (4 / 8 per lane), 8 / 9 the
                                same in XCD runs; 10 / 11 2 / 1 per lane in XCD runs of 4
                                blocks, 12 2 per lane without runs, 13 2 per lane in runs of 8 */
    int32_t rg_p1;           /* row-segment pass 1: 0 / 1 by groups (2^k lanes per group, DPP
                                merges), 2 evenly split runs (NT / groups lanes per group, LDS
                                merges, parameters by one lane per group) */
    int32_t rg_lds_full;     /* row-segment LDS stage: 0 sized to the elements a tile holds (min(groups
                                x group size, K)), 1 to its groups x group size (round-2 sizing, A/B) */
    int32_t rg_ldsdma;       /* row-segment stage: 0 LDS-DMA (buffer_load_dwordx4 ... lds, the default),
                                1 the round-3 register stage (loads to VGPRs, LDS stores) */
    int32_t rg_p2reg;        /* with rg_ldsdma = 1: pass 2 of a 4-chunk stage from the stage's
                                registers (0) or from LDS (1) */
    int32_t rg_p1u;          /* row-segment pass 1: 0 the uniform form where it applies (round 4),
                                1 always the per-lane bounds form (A/B) */
} awq_tuning;

#ifdef AWQ_DIAG
/* Set (t != NULL) or reset to the defaults (t == NULL) this thread's tuning. */
int awq_set_tuning(const awq_tuning* t);
#endif

#ifdef __cplusplus
}
#endif
#endif /* AWQ_DIAG_H */
