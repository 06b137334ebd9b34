/*
 * nkfs_crt.h -- the drop-in C-ABI of libnkfs_crt.so (MI355X / gfx950).
 *
 * These are the reference's own crt/ symbols for the erasure-code and
 * checksum path, unchanged in name, argument meaning, ownership and error
 * behaviour, so that a caller built against irqlevel/nkfs crt/ links
 * against libnkfs_crt.so instead of nkfs_crtlib.a.  Every computation behind
 * them runs on the GPU (HIP kernels in nkfs_amd/csrc/nk8_kernels.hip); the
 * host side only validates, moves bytes and keeps state.  Without a usable
 * GPU nk8_init() fails with -ENODEV and every compute entry point fails
 * loudly -- there is no CPU fallback.
 *
 * Batched, device-resident entry points (explicit ids, device pointers,
 * streams) are in nkfs_gpu.h.
 */
#ifndef NKFS_CRT_H
#define NKFS_CRT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------- nk8 code */

/* replaces crt/include/nk8.h:4 (crt/nk8.c:725-747).  Selects the GPU
 * (env NKFS_DEVICE, default the current HIP device), builds the GF(2^8)
 * tables on it and runs the reference's load-time self test (five random
 * split -> k-of-n assemble round trips compared by XXH64) on the GPU.
 * 0, or -ENODEV (no GPU), -EIO (HIP failure), or the self-test error. */
int nk8_init(void);

/* replaces crt/include/nk8.h:5 (crt/nk8.c:749-752): releases device state. */
void nk8_release(void);

/* replaces crt/include/nk8.h:7-8 (crt/nk8.c:344-444).  Encodes block into n
 * parts of ceil(block_size/k) bytes with n random distinct ids in 1..255
 * (the reference's rule, crt/nk8.c:319-342).  The callee allocates
 * *pparts (n pointers), every part and *pids with crt_malloc; the caller
 * frees them with crt_free.  -EINVAL (2<=k<=n, k<=254, n<=255,
 * block_size>0 violated), -EAGAIN before nk8_init, -ENOMEM, -EIO. */
int nk8_split_block(uint8_t *block, uint32_t block_size, int n, int k,
		    uint8_t ***pparts, uint8_t **pids);

/* replaces crt/include/nk8.h:10-11 (crt/nk8.c:446-599).  Rebuilds block
 * (exactly block_size bytes) from the FIRST k parts whose ids are distinct,
 * in argument order; later parts are ignored.  -EINVAL if fewer than k
 * distinct ids or bad params, -EAGAIN before nk8_init, -EFAULT singular. */
int nk8_assemble_block(uint8_t **parts, uint8_t *ids, int n, int k,
		       uint8_t *block, uint32_t block_size);

/* --------------------------------------------------------------- XXH64 */

/* crt/include/xxhash.h:77 */
typedef enum { XXH_OK = 0, XXH_ERROR } XXH_errorcode;
/* crt/include/xxhash.h:105 -- opaque, 88 bytes; the internal layout is the
 * reference's XXH_istate64_t (crt/xxhash.c:515-525) so states embedded in
 * callers' structs (struct csum_ctx) keep their size. */
typedef struct { long long ll[11]; } XXH64_state_t;

/* crt/include/xxhash.h:86 */
unsigned long long XXH64(const void *input, size_t length, unsigned long long seed);
/* crt/include/xxhash.h:117-118 */
XXH64_state_t *XXH64_createState(void);
XXH_errorcode XXH64_freeState(XXH64_state_t *state);
/* crt/include/xxhash.h:130-132 */
XXH_errorcode XXH64_reset(XXH64_state_t *state, unsigned long long seed);
XXH_errorcode XXH64_update(XXH64_state_t *state, const void *input, size_t length);
unsigned long long XXH64_digest(const XXH64_state_t *state);

/* ---------------------------------------------------------------- csum */

/* crt/include/csum.h:6-12 */
struct csum {
	uint64_t val;
};
struct csum_ctx {
	XXH64_state_t state;
};

/* crt/include/csum.h:14-17 (crt/csum.c:3-27): XXH64 with seed 0; a failed
 * step traps like the reference's CRT_BUG (crt/user/crt.h:32-33). */
void csum_reset(struct csum_ctx *ctx);
void csum_update(struct csum_ctx *ctx, const void *input, size_t len);
void csum_digest(struct csum_ctx *ctx, struct csum *sum);
uint64_t csum_u64(struct csum *sum);

/* ------------------------------------------------------------- memory */

/* crt/include/crt.h:12-13 (crt/user/crt.c:150-173): split's outputs are
 * crt_malloc'd host memory the caller releases with crt_free. */
void *crt_malloc(size_t size);
void crt_free(void *ptr);

#ifdef __cplusplus
}
#endif
#endif
