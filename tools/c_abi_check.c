/* tools/c_abi_check.c — a plain C11 consumer of the C-ABI headers (no C++, no HIP headers): proves
 * that the include/dccl headers are valid C and that libdccl_amd.so links from C, as a DCCL-side FFI caller
 * would use it.  Without arguments it runs the checks that need no GPU; with "gpu" it also runs the
 * host-pointer combine (staged through the current GPU) against a plain C loop.
 *
 *   gcc -std=c11 -Wall -Wextra -pedantic -Werror -I include tools/c_abi_check.c \
 *       -L dccl_amd/lib -ldccl_amd -Wl,-rpath,dccl_amd/lib -o dccl_amd/bin/c_abi_check
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dccl/dccl_comm.h"
#include "dccl/dccl_reduce.h"
#include "dccl/dccl_synth.h"

static int failures = 0;

#define CHECK(cond)                                                      \
    do {                                                                 \
        if (!(cond)) {                                                   \
            fprintf(stderr, "c_abi_check: %s:%d: %s\n", __FILE__, __LINE__, #cond); \
            failures++;                                                  \
        }                                                                \
    } while (0)

static void cpu_checks(void) {
    static const size_t sizes[10] = {1, 1, 4, 4, 8, 8, 2, 4, 8, 2};
    for (int t = 0; t < 10; ++t) CHECK(dccl_size_of_type(t) == sizes[t]);
    CHECK(dccl_size_of_type(10) == 0);
    CHECK(dccl_version() > 0);
    CHECK(strlen(dccl_result_string(DCCL_SUCCESS)) > 0);
    float a[4] = {0}, b[4] = {0};
    /* argument validation happens before any device work */
    CHECK(dccl_local_reduce(a, b, 7, 4, 4, NULL) == DCCL_INVALID_USAGE);    /* ncclAvg */
    CHECK(dccl_local_reduce(a, b, 7, 4, 9, NULL) == DCCL_INVALID_ARGUMENT); /* bad op */
    CHECK(dccl_local_reduce(a, b, 11, 4, 0, NULL) == DCCL_INVALID_ARGUMENT); /* bad dtype */
    CHECK(dccl_local_reduce(a, b, 7, 0, 0, NULL) == DCCL_SUCCESS);          /* count 0 */
    CHECK(dccl_local_reduce_host(a, b, 7, 4, 4) == DCCL_INVALID_USAGE);
    const void* sends[1] = {a};
    CHECK(dccl_local_reduce_multi(sends, 0, b, 7, 4, 0, NULL) == DCCL_INVALID_ARGUMENT);
    CHECK(dccl_local_reduce_chain(sends, 9, a, b, 7, 4, 0, NULL) == DCCL_INVALID_ARGUMENT);
    CHECK(dccl_local_reduce_chain_host(sends, 0, a, b, 7, 4, 0) == DCCL_INVALID_ARGUMENT);
    CHECK(dccl_synth_fill(NULL, 7, 16, 0, 1, 0, NULL) == DCCL_INVALID_ARGUMENT);
    CHECK(dccl_copy_multi(NULL, NULL, 0, 16, NULL) == DCCL_SUCCESS);
    CHECK(dccl_all_reduce(a, b, 4, 7, 0, NULL, NULL) == DCCL_INVALID_ARGUMENT); /* null communicator */
    /* partial overlap with the destination (one element apart) is rejected before any device work */
    float c[8] = {0};
    CHECK(dccl_local_reduce(c + 1, c, 7, 4, 0, NULL) == DCCL_INVALID_ARGUMENT);
    CHECK(dccl_local_reduce_host(c, c + 1, 7, 4, 0) == DCCL_INVALID_ARGUMENT);
    const void* ov[1] = {c + 1};
    CHECK(dccl_local_reduce_multi(ov, 1, c, 7, 4, 0, NULL) == DCCL_INVALID_ARGUMENT);
    CHECK(dccl_local_reduce_chain(sends, 1, c + 3, c, 7, 4, 0, NULL) == DCCL_INVALID_ARGUMENT);
    CHECK(dccl_local_reduce_chain_host(ov, 1, a, c, 7, 4, 0) == DCCL_INVALID_ARGUMENT);
    /* routing hint: the reference has no host loop for bf16 / fp16 */
    CHECK(dccl_host_reduce_gpu_min_bytes(9) == 0 && dccl_host_reduce_gpu_min_bytes(6) == 0);
}

static void gpu_checks(void) {
    enum { N = 100003 };
    float* s = malloc(N * sizeof(float));
    float* r = malloc(N * sizeof(float));
    float* want = malloc(N * sizeof(float));
    int8_t* si = malloc(N);
    int8_t* ri = malloc(N);
    int8_t* wanti = malloc(N);
    if (!s || !r || !want || !si || !ri || !wanti) {
        failures++;
        return;
    }
    for (int i = 0; i < N; ++i) {
        s[i] = (float)(i % 977) * 0.25f - 100.0f;
        r[i] = (float)(i % 131) * 0.5f;
        want[i] = r[i] + s[i];
        si[i] = (int8_t)(i * 7);
        ri[i] = (int8_t)(i * 13 + 1);
        wanti[i] = (int8_t)(ri[i] * si[i]); /* wraps, like the reference's int8 r *= s */
    }
    CHECK(dccl_local_reduce_host(s, r, 7, N, 0) == DCCL_SUCCESS);
    CHECK(memcmp(r, want, N * sizeof(float)) == 0);
    CHECK(dccl_local_reduce_host(si, ri, 0, N, 1) == DCCL_SUCCESS);
    CHECK(memcmp(ri, wanti, N) == 0);
    free(s), free(r), free(want), free(si), free(ri), free(wanti);
}

int main(int argc, char** argv) {
    cpu_checks();
    if (argc > 1 && strcmp(argv[1], "gpu") == 0) gpu_checks();
    printf("c_abi_check: %s\n", failures ? "FAILED" : "ok");
    return failures ? 1 : 0;
}
