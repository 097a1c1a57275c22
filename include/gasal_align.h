/*
 * gasal_align.h — asynchronous alignment entry points.
 * Replaces Non-CDP/GASAL2/src/gasal_align.h:114-120 (the macro kernel switch
 * at :7-107 is replaced by the flat host dispatcher in
 * genomics-gpu_amd/csrc/dispatch.hip).
 */
#ifndef __GASAL_ALIGN_H__
#define __GASAL_ALIGN_H__

#include "gasal.h"
#include "args_parser.h"

/* gasal_align.cu:329-339: scores become kernel arguments of the current device. */
void gasal_copy_subst_scores(gasal_subst_scores *subst);

/* gasal_align.cu:29-307 */
void gasal_aln_async(gasal_gpu_storage_t *gpu_storage, const uint32_t actual_query_batch_bytes,
                     const uint32_t actual_target_batch_bytes, const uint32_t actual_n_alns,
                     Parameters *params);

/* gasal_align.cu:310-326: 0 done, -1 busy, -2 nothing launched. */
int gasal_is_aln_async_done(gasal_gpu_storage_t *gpu_storage);

#endif
