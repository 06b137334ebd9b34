/*
 * csum.c -- the reference's checksum ABI (crt/include/csum.h:14-17,
 * crt/include/xxhash.h:86-132; XXH32 is not on the path and not exported)
 * with the XXH64 rounds, merge, tail and avalanche computed on the GPU
 * (k_xxh64_stripes / k_xxh64_finish in nk8_kernels.hip).
 *
 * The state keeps the reference's internal layout (crt/xxhash.c:515-525)
 * inside the caller-owned 88-byte XXH64_state_t, and the host side does what
 * the reference's update does with memory: it buffers an incomplete 32-byte
 * stripe in mem64 (crt/xxhash.c:750-770, 823-833).  Each update that
 * completes at least one stripe ships the stripes and the four accumulators
 * to the device, folds them there and brings the accumulators back.
 *
 * These per-call entry points keep drop-in callers (client/lib/client.c,
 * crt/net_pkt.c) working; high-volume hashing belongs in
 * nkfs_xxh64_batch / the fused encode (include/nkfs_gpu.h).
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/nkfs_crt.h"
#include "../../include/nkfs_gpu.h"
#include "nkfs_internal.h"
#include "runtime.h"

struct xstate {           /* crt/xxhash.c:515-525 */
	uint64_t total_len;
	uint64_t seed;
	uint64_t v[4];
	uint64_t mem64[4];
	uint32_t memsize;
};
_Static_assert(sizeof(struct xstate) <= sizeof(XXH64_state_t), "XXH64_state_t too small");

#define P1 0x9E3779B185EBCA87ULL
#define P2 0xC2B2AE3D27D4EB4FULL

static int ensure_gpu(void)
{
	return nkfs_gpu_ready() ? 0 : nkfs_gpu_init(-1);
}

XXH64_state_t *XXH64_createState(void)
{
	return crt_malloc(sizeof(XXH64_state_t));
}

XXH_errorcode XXH64_freeState(XXH64_state_t *state)
{
	crt_free(state);
	return XXH_OK;
}

XXH_errorcode XXH64_reset(XXH64_state_t *state_in, unsigned long long seed)
{
	struct xstate *s = (struct xstate *)state_in;
	s->seed = seed;
	s->v[0] = seed + P1 + P2;
	s->v[1] = seed + P2;
	s->v[2] = seed;
	s->v[3] = seed - P1;
	s->total_len = 0;
	s->memsize = 0;
	return XXH_OK;
}

/* Stripes per device pass: the input streams through bounded pinned and
 * device scratch (8 MiB + the state), so any length hashes without a
 * device allocation of its size. */
#define FOLD_CHUNK (8u << 20)

/* Fold the buffered stripe (if `lead`) and `nst_input` stripes of the
 * caller's bytes into s->v on the device: state + stripes are staged in
 * pinned memory and go over in one copy per chunk; the accumulators stay
 * on the device between chunks and come back once. */
static int fold_stripes(struct xstate *s, const uint8_t *lead, const uint8_t *input, uint64_t nst_input)
{
	struct nkfs_ctx *c = nkfs_ctx_get();
	if (!c)
		return -EIO;
	int err;
	const uint64_t total = (lead ? 1 : 0) + nst_input;  /* stripes */
	const uint64_t first = total * 32 < FOLD_CHUNK ? total * 32 : FOLD_CHUNK;
	void *dv, *hv;
	if ((err = nkfs_ctx_dev(c, 64 + first, &dv)) || (err = nkfs_ctx_host(c, 64 + first, &hv)))
		goto out;
	uint8_t *d = dv, *h = hv;
	memcpy(h, s->v, 32);
	uint64_t done = 0;  /* input stripes consumed */
	for (int pass = 0; done < nst_input || (pass == 0 && lead); pass++) {
		uint64_t off = pass == 0 ? 32 : 0; /* pass 0 carries the state */
		uint64_t room = (FOLD_CHUNK - (pass == 0 && lead ? 32 : 0)) / 32;
		uint64_t take = nst_input - done < room ? nst_input - done : room;
		uint8_t *hp = h + 32;
		if (pass == 0 && lead) {
			memcpy(hp, lead, 32);
			hp += 32;
		}
		if (pass) /* the previous pass's copy must be done before the staging is reused */
			if (hipStreamSynchronize(c->stream) != hipSuccess) {
				err = -EIO;
				goto out;
			}
		memcpy(hp, input + done * 32, take * 32);
		const uint64_t nst = take + (pass == 0 && lead ? 1 : 0);
		if (hipMemcpyAsync(d + 32 - off, h + 32 - off, off + nst * 32, hipMemcpyHostToDevice, c->stream) !=
		    hipSuccess) {
			err = -EIO;
			goto out;
		}
		if ((err = nkfs_launch_xxh64_stripes((uint64_t *)d, d + 32, nst, c->stream)))
			goto out;
		done += take;
	}
	if (hipMemcpyAsync(h, d, 32, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
	    hipStreamSynchronize(c->stream) != hipSuccess) {
		err = -EIO;
		goto out;
	}
	memcpy(s->v, h, 32);
out:
	nkfs_ctx_put(c);
	return err;
}

XXH_errorcode XXH64_update(XXH64_state_t *state_in, const void *input, size_t len)
{
	struct xstate *s = (struct xstate *)state_in;
	const uint8_t *p = input;
	if (!input && len)
		return XXH_ERROR;
	if (s->memsize + len < 32) {
		if (len)
			memcpy((uint8_t *)s->mem64 + s->memsize, p, len);
		s->memsize += (uint32_t)len;
		s->total_len += len;
		return XXH_OK;
	}
	if (ensure_gpu())
		return XXH_ERROR;
	const uint8_t *lead = NULL;
	if (s->memsize) {
		size_t fill = 32 - s->memsize;
		memcpy((uint8_t *)s->mem64 + s->memsize, p, fill);
		p += fill;
		len -= fill;
		s->total_len += fill;
		lead = (const uint8_t *)s->mem64;
		s->memsize = 0;
	}
	uint64_t nst = len / 32;
	if (lead || nst) {
		if (fold_stripes(s, lead, p, nst))
			return XXH_ERROR;
	}
	p += nst * 32;
	len -= nst * 32;
	s->total_len += nst * 32;
	memcpy(s->mem64, p, len);
	s->memsize = (uint32_t)len;
	s->total_len += len;
	return XXH_OK;
}

/* returns 0 and fills *out, or a negative errno */
static int finish(const struct xstate *s, uint64_t *out)
{
	if (ensure_gpu())
		return -ENODEV;
	struct nkfs_ctx *c = nkfs_ctx_get();
	if (!c)
		return -EIO;
	int err;
	void *dv, *hv;
	if ((err = nkfs_ctx_dev(c, 80, &dv)) || (err = nkfs_ctx_host(c, 80, &hv)))
		goto out;
	uint8_t *d = dv, *h = hv;
	memcpy(h, s->v, 32);
	memcpy(h + 32, s->mem64, 32);
	if (hipMemcpyAsync(d, h, 64, hipMemcpyHostToDevice, c->stream) != hipSuccess) {
		err = -EIO;
		goto out;
	}
	if ((err = nkfs_launch_xxh64_finish((uint64_t *)(d + 64), (const uint64_t *)d, s->total_len, s->seed, d + 32,
					    s->memsize, c->stream)))
		goto out;
	if (hipMemcpyAsync(h + 64, d + 64, 8, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
	    hipStreamSynchronize(c->stream) != hipSuccess) {
		err = -EIO;
		goto out;
	}
	memcpy(out, h + 64, 8);
out:
	nkfs_ctx_put(c);
	return err;
}

/* The reference returns a digest unconditionally; a GPU failure here has
 * no error channel, so it traps like CRT_BUG rather than return a wrong
 * checksum. */
unsigned long long XXH64_digest(const XXH64_state_t *state_in)
{
	uint64_t h;
	if (finish((const struct xstate *)state_in, &h))
		__builtin_trap();
	return h;
}

unsigned long long XXH64(const void *input, size_t length, unsigned long long seed)
{
	XXH64_state_t st;
	XXH64_reset(&st, seed);
	if (XXH64_update(&st, input, length) != XXH_OK)
		__builtin_trap();
	return XXH64_digest(&st);
}

/* crt/csum.c:3-27 */
void csum_reset(struct csum_ctx *ctx)
{
	if (XXH64_reset(&ctx->state, 0))
		__builtin_trap();
}

void csum_update(struct csum_ctx *ctx, const void *input, size_t len)
{
	if (XXH64_update(&ctx->state, input, len))
		__builtin_trap();
}

void csum_digest(struct csum_ctx *ctx, struct csum *sum)
{
	sum->val = XXH64_digest(&ctx->state);
}

uint64_t csum_u64(struct csum *sum)
{
	return sum->val;
}
