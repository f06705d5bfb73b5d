// sddc_ddc_internal.h — development-only entry points (not part of the C ABI contract).
#pragma once
#include "sddc_ddc.h"
#ifdef __cplusplus
extern "C" {
#endif
/* A tuning parameter of the kernels (A/B timing, tools/ab_libs.py --param):
 * SDDC_DDC_PARAM_FS_STATIC_PCT = the d = 0 kernel's share of each workgroup's frames taken
 * statically before it draws from the dynamic queue (0..100, default kFsStaticPct). */
#define SDDC_DDC_PARAM_FS_STATIC_PCT 1
/* SDDC_DDC_PARAM_SLOT_WEIGHTS = 1: the persistent kernel splits the frames by CU slot speed
 * (kSlotWeights[d]), 0: equal contiguous ranges (default kSlotWeighting). */
#define SDDC_DDC_PARAM_SLOT_WEIGHTS 2
/* SDDC_DDC_PARAM_FS_FRAMES_PER_WG = n > 0: the d = 0 kernel runs a non-persistent grid of
 * ceil(frames / n) workgroups, n frames each, balanced by the hardware dispatcher; 0 (default):
 * the persistent grid. */
#define SDDC_DDC_PARAM_FS_FRAMES_PER_WG 3
/* SDDC_DDC_PARAM_FS_SCHEDULE: the d = 0 kernel's frame schedule, 0 = the slot-weighted static
 * split alone (default), 1 = static prefix + dynamic queue, 2 = work stealing (1 and 2 only for
 * CF32 output without NCO, rand or sideband inversion; other configurations fail to launch). */
#define SDDC_DDC_PARAM_FS_SCHEDULE 4
/* SDDC_DDC_PARAM_FS_STEAL_MINREM: a thief steals only from ranges with at least this many
 * unclaimed frames (1..64; 0: no stealing, the static split inside the stealing kernel). */
#define SDDC_DDC_PARAM_FS_STEAL_MINREM 5
/* SDDC_DDC_PARAM_FS_STEAL_PUBLIC: frames at the end of each workgroup's range open to thieves,
 * claimed by the owner with atomics (0: all but the first two); the rest the owner takes alone. */
#define SDDC_DDC_PARAM_FS_STEAL_PUBLIC 6
/* SDDC_DDC_PARAM_FS_ZERO_ROWS != 0 (default 1): the d = 0 kernel skips the inverse input's whole
 * zero rows of the tune bin (ddc_fs.hip fs_zero_rows: 2..8 rows for CF32 output without the NCO,
 * 4 rows or none for the fused-NCO and CS16 outputs and the queue / stealing schedules; a single
 * zero row is computed); 0: computes them all (A/B, tests). */
#define SDDC_DDC_PARAM_FS_ZERO_ROWS 7
/* SDDC_DDC_PARAM_FS_SLOT_WEIGHTS: the d = 0 kernel's slot weights of the static split, four
 * bytes w0 | w1 << 8 | w2 << 16 | w3 << 24 (CU slot 0 in the low byte, each 1..127); 0: the
 * built-in kFsSlotWeights (A/B of the weights). */
#define SDDC_DDC_PARAM_FS_SLOT_WEIGHTS 8

int sddc_ddc_internal_set_param(sddc_ddc_t *h, int param, int value);
/* Diagnostic stamp buffers of -DSDDC_STAMPS builds (tools/fs_stamps.py); -1 in product builds. */
int sddc_ddc_internal_fs_stamps(unsigned *host, int nwords, int *words_per_wave);
int sddc_ddc_internal_p_stamps(unsigned *host, int nwords, int *words_per_wave);
#ifdef __cplusplus
}
#endif
