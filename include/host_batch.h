/* host_batch.h — extensible pinned host pages, drop-in for Non-CDP/GASAL2/src/host_batch.h:1-20. */
#ifndef __HOST_BACTH_H__
#define __HOST_BACTH_H__

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gasal.h"

host_batch_t *gasal_host_batch_new(uint32_t batch_bytes, uint32_t offset);
void gasal_host_batch_destroy(host_batch_t *res);
host_batch_t *gasal_host_batch_getlast(host_batch_t *arg);
void gasal_host_batch_reset(gasal_gpu_storage_t *gpu_storage);
uint32_t gasal_host_batch_fill(gasal_gpu_storage_t *gpu_storage, uint32_t idx, const char *data, uint32_t size,
                               data_source SRC);
uint32_t gasal_host_batch_add(gasal_gpu_storage_t *gpu_storage, uint32_t idx, const char *data, uint32_t size,
                              data_source SRC);
uint32_t gasal_host_batch_addbase(gasal_gpu_storage_t *gpu_storage, uint32_t idx, const char base, data_source SRC);
void gasal_host_batch_print(host_batch_t *res);
void gasal_host_batch_printall(host_batch_t *res);

#endif
