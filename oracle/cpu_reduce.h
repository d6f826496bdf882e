/* cpu_reduce.h — ORACLE / TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of Gloo's per-chunk reduction (gloo/math.h:15-73) used
 * as the parity checker for the HIP kernels.  Never linked into gloo_amd/;
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it.  Op / dtype codes are those of include/gloo_amd.h.
 *
 * Pinned by tests/test_oracle.py against the golden vectors in tests/golden/
 * that oracle/gen_golden.py generated from the reference itself
 * (oracle/_ref/libgloo_ref.so, built from /root/reference by oracle/Makefile).
 */
#ifndef GLOO_ORACLE_CPU_REDUCE_H_
#define GLOO_ORACLE_CPU_REDUCE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* c[i] = a[i] (op) b[i] for i < n, in index order (c may alias a or b). */
int oracle_reduce3(int op, int dtype, void* c, const void* a, const void* b, size_t n);

/* dst = ((srcs[0] op srcs[1]) op srcs[2]) ... (gloo/allreduce_local.cc:28-33). */
int oracle_reduce_multi(int op, int dtype, void* dst, const void* const* srcs, int k,
                        size_t n);

/* Scalar conversions used by the fp16 / bf16 paths (exposed for tests). */
uint16_t oracle_f32_to_f16(float f);
float oracle_f16_to_f32(uint16_t h);
uint16_t oracle_f32_to_bf16(float f);
float oracle_bf16_to_f32(uint16_t h);

/* fp32 SUM over `nthreads` host threads (CPU baseline when oracle/_ref is
 * unavailable); nthreads <= 1 is the single-threaded loop gloo runs. */
void oracle_sum_f32_mt(float* c, const float* a, const float* b, size_t n, int nthreads);

#ifdef __cplusplus
}
#endif

#endif
