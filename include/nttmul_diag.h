/*
 * nttmul_diag.h — the diagnostic build lib/libnttmul_diag.so (not libnttmul.so).
 *
 * Same C ABI and the same product kernels as include/nttmul.h, built with NTTMUL_CLOCK_STAMPS:
 * thread 0 of every k_rows workgroup (the fused product at n <= 4096, the row pass above)
 * stamps s_memtime and s_memrealtime at entry and after issuing its stores, so a caller can read
 * the shader clock the product kernel actually held (MI355X_MICROARCH.md 'DVFS give-back' item 6)
 * — bench.py puts it beside the VALU issue bound.  The stamps go to a buffer of their own; no
 * output depends on them.  The production library executes no stamp.
 */
#ifndef NTTMUL_DIAG_H
#define NTTMUL_DIAG_H

#include "nttmul.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The last k_rows launch's stamps of workgroups 0 .. blocks - 1 (at most 65536), four uint64 per
 * workgroup: entry s_memtime, entry s_memrealtime, end s_memtime, end s_memrealtime.  The
 * workgroup's clock is (end_t - entry_t) / (end_r - entry_r) x 100 MHz.  Call after the launch
 * has completed. */
int nttmul_diag_clock_stamps(uint64_t *dst, size_t blocks);

/* The resident device server's timeline of ctx's last host product served through it
 * (nttmul_last_host_path == 3; params.small_server): dst[0..3] = s_memrealtime (100 MHz) when
 * the kernel saw the request, had a and b loaded, had the product computed, had c stored and
 * released; dst[4], dst[5] = s_memtime (shader clock) around the product; dst[6] = host
 * nanoseconds from posting the request to seeing it done.  NTTMUL_EINVAL if the last call did not
 * go through the server. */
int nttmul_diag_server_stamps(const nttmul_ctx *ctx, uint64_t *dst);

#ifdef __cplusplus
}
#endif

#endif /* NTTMUL_DIAG_H */
