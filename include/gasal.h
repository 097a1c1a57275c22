/*
 * gasal.h — public types of the MI355X GASAL2-compatible alignment engine.
 *
 * Drop-in for Non-CDP/GASAL2/src/gasal.h:1-168 (reference).  Names, enum
 * values and struct field order are identical so that code written against the
 * reference (e.g. test_prog.cpp) compiles unchanged; the only substitution is
 * cudaStream_t -> hipStream_t (both opaque pointers, same layout).  The
 * reference's error helpers keep their names (CHECKCUDAERROR assigns to the
 * caller's `err`, as gasal.h:15-22 does; CudaCheckKernelLaunch, :25-34) and
 * check HIP status codes; CHECKHIPERROR is the self-contained form.  uint4 comes
 * from the HIP vector types.
 */
#ifndef __GASAL_H__
#define __GASAL_H__

#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

#include <hip/hip_runtime_api.h>
#include <hip/hip_vector_types.h>

#ifndef HOST_MALLOC_SAFETY_FACTOR
#define HOST_MALLOC_SAFETY_FACTOR 5
#endif

/* gasal.h:15-22 — print and exit on any runtime error. */
#define CHECKHIPERROR(error)                                                                 \
    do {                                                                                     \
        hipError_t gasal_err__ = (error);                                                    \
        if (hipSuccess != gasal_err__) {                                                     \
            fprintf(stderr, "[GASAL HIP ERROR:] %s(HIP error no.=%d). Line no. %d in file %s\n", \
                    hipGetErrorString(gasal_err__), (int)gasal_err__, __LINE__, __FILE__);   \
            exit(EXIT_FAILURE);                                                              \
        }                                                                                    \
    } while (0)

/* gasal.h:15-22 under its own name: `err` is the caller's status variable (hipError_t). */
#define CHECKCUDAERROR(error)                                                                \
    do {                                                                                     \
        err = (error);                                                                       \
        if (hipSuccess != err) {                                                             \
            fprintf(stderr, "[GASAL CUDA ERROR:] %s(CUDA error no.=%d). Line no. %d in file %s\n", \
                    hipGetErrorString(err), (int)err, __LINE__, __FILE__);                   \
            exit(EXIT_FAILURE);                                                              \
        }                                                                                    \
    } while (0)

/* gasal.h:25-34: -1 when the last launch failed. */
inline int CudaCheckKernelLaunch() {
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

enum comp_start {
    WITHOUT_START,
    WITH_START,
    WITH_TB
};

enum Bool {
    FALSE,
    TRUE
};

enum data_source {
    NONE,
    QUERY,
    TARGET,
    BOTH
};

enum algo_type {
    UNKNOWN,
    GLOBAL,
    SEMI_GLOBAL,
    LOCAL,
    MICROLOCAL,
    BANDED,
    KSW
};

enum operation_on_seq {
    FORWARD_NATURAL,
    REVERSE_NATURAL,
    FORWARD_COMPLEMENT,
    REVERSE_COMPLEMENT,
};

/* Extensible chain of pinned host pages (gasal.h:75-83). */
struct host_batch {
    uint8_t *data;
    uint32_t page_size;
    uint32_t data_size;
    uint32_t offset;
    int is_locked;
    struct host_batch *next;
};
typedef struct host_batch host_batch_t;

/* Result arrays, host- or device-resident (gasal.h:85-95). */
struct gasal_res {
    int32_t *aln_score;
    int32_t *query_batch_end;
    int32_t *target_batch_end;
    int32_t *query_batch_start;
    int32_t *target_batch_start;
    uint8_t *cigar;
    uint32_t *n_cigar_ops;
};
typedef struct gasal_res gasal_res_t;

/* Per-stream storage (gasal.h:97-152).  Field order is the reference's. */
typedef struct {
    uint8_t *unpacked_query_batch;
    uint8_t *unpacked_target_batch;
    uint32_t *packed_query_batch;
    uint32_t *packed_target_batch;
    uint32_t *query_batch_offsets;
    uint32_t *target_batch_offsets;
    uint32_t *query_batch_lens;
    uint32_t *target_batch_lens;

    uint32_t *host_seed_scores;
    uint32_t *seed_scores;

    host_batch_t *extensible_host_unpacked_query_batch;
    host_batch_t *extensible_host_unpacked_target_batch;

    uint8_t *host_query_op;
    uint8_t *host_target_op;
    uint8_t *query_op;
    uint8_t *target_op;

    uint32_t *host_query_batch_offsets;
    uint32_t *host_target_batch_offsets;
    uint32_t *host_query_batch_lens;
    uint32_t *host_target_batch_lens;

    gasal_res_t *host_res;
    gasal_res_t *device_cpy;
    gasal_res_t *device_res;

    gasal_res_t *host_res_second;
    gasal_res_t *device_res_second;
    gasal_res_t *device_cpy_second;

    uint32_t gpu_max_query_batch_bytes;
    uint32_t gpu_max_target_batch_bytes;

    uint32_t host_max_query_batch_bytes;
    uint32_t host_max_target_batch_bytes;

    uint32_t gpu_max_n_alns;
    uint32_t host_max_n_alns;
    uint32_t current_n_alns;

    uint64_t packed_tb_matrix_size;
    uint4 *packed_tb_matrices;

    hipStream_t str;
    int is_free;
    int id;

} gasal_gpu_storage_t;

typedef struct {
    int n;
    gasal_gpu_storage_t *a;
} gasal_gpu_storage_v;

typedef struct {
    int32_t match;
    int32_t mismatch;
    int32_t gap_open;
    int32_t gap_extend;
} gasal_subst_scores;

#endif
