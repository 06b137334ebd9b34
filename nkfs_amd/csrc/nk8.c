/*
 * nk8.c -- the reference's nk8_* entry points (crt/include/nk8.h:4-11) on
 * the MI355X.  Same names, argument meaning, ownership (callee crt_mallocs,
 * caller crt_frees) and error codes as crt/nk8.c; the encode, the decode and
 * the K x K inverse run as HIP kernels (nk8_kernels.hip, nk8_fast.hip) on a
 * per-call context from runtime.c.  The host side validates arguments,
 * draws part ids, picks the parts to upload and moves bytes.
 */
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/random.h>
#include <unistd.h>

#include "../../include/nkfs_crt.h"
#include "../../include/nkfs_gpu.h"
#include "nkfs_internal.h"
#include "runtime.h"

static int nk8_inited;

static int rand_bytes(void *buf, size_t len)
{
	uint8_t *p = buf;
	while (len) {
		ssize_t r = getrandom(p, len, 0);
		if (r < 0) {
			if (errno == EINTR)
				continue;
			return -errno;
		}
		p += r;
		len -= (size_t)r;
	}
	return 0;
}

/* getrandom bytes drawn 256 at a time per thread: a drop-in split draws n
 * ids, one 8-byte word each (more on rejection), and a syscall per word
 * cost microseconds of a ~15 us call.  The words are the same uniform bytes
 * (crt/random.c draws from getrandom as well).  The pool is tagged with the
 * pid that filled it: a forked child refills instead of handing out its
 * parent's next words (the reference draws fresh bytes per call). */
static __thread uint8_t g_rpool[256];
static __thread unsigned g_rpos = sizeof(g_rpool);
static __thread pid_t g_rpid;

static int rand_word(uint64_t *out)
{
	const pid_t me = getpid();
	if (g_rpid != me) {
		g_rpid = me;
		g_rpos = sizeof(g_rpool);
	}
	if (g_rpos + sizeof(*out) > sizeof(g_rpool)) {
		int err = rand_bytes(g_rpool, sizeof(g_rpool));
		if (err)
			return err;
		g_rpos = 0;
	}
	memcpy(out, g_rpool + g_rpos, sizeof(*out));
	memset(g_rpool + g_rpos, 0, sizeof(*out)); /* a word is used once */
	g_rpos += sizeof(*out);
	return 0;
}

/* uniform in [0, up) by rejection on the next power of two, as
 * rand_u32_up (crt/random.c:15-33) */
static int rand_below(uint32_t up, uint32_t *out)
{
	uint32_t bits = 0;
	while ((1u << bits) < up)
		bits++;
	for (;;) {
		uint64_t r;
		int err = rand_word(&r);
		if (err)
			return err;
		uint32_t v = (uint32_t)(r & ((1ull << bits) - 1));
		if (v < up) {
			*out = v;
			return 0;
		}
	}
}

/* n distinct ids in 1..255 (crt/nk8.c:319-342) */
static int gen_part_ids(uint8_t *ids, int n)
{
	for (int i = 0; i < n; i++) {
		for (;;) {
			uint32_t v;
			int err = rand_below(255, &v);
			if (err)
				return err;
			uint8_t cand = (uint8_t)(1 + v);
			int dup = 0;
			for (int j = 0; j < i; j++)
				dup |= ids[j] == cand;
			if (!dup) {
				ids[i] = cand;
				break;
			}
		}
	}
	return 0;
}

#define HIPGO(call)                                                              \
	do {                                                                     \
		hipError_t e_ = (call);                                          \
		if (e_ != hipSuccess) {                                          \
			err = nkfs_hip_fail(#call, (int)e_);                     \
			goto out;                                                \
		}                                                                \
	} while (0)

static uint64_t round16(uint64_t v) { return (v + 15) & ~(uint64_t)15; }

/* Encode one block on the GPU with explicit ids into host part buffers.
 * Block and ids go over in one copy from pinned staging, the n parts come
 * back in one copy (the per-call fixed cost is two copies, one launch and
 * one stream sync). */
/* Blocks up to this size take the zero-copy form: the kernel reads the
 * block from the pinned staging buffer and writes the parts back into it
 * over PCIe, so a small call costs one launch and one sync instead of two
 * DMA copies as well. */
#ifndef NKFS_ZC_MAX
#define NKFS_ZC_MAX 1048576
#endif
/* blocks from this size wait by spinning on a completion word (nkfs_ctx_wait) */
#define NKFS_SPIN_MIN 32768

static int gpu_split(const uint8_t *block, uint32_t B, int n, int k, const uint8_t *ids, uint8_t **parts)
{
	struct nkfs_ctx *c = nkfs_ctx_get();
	if (!c)
		return -EIO;
	int err;
	uint32_t ps = nkfs_part_size(B, k);
	uint64_t pitch = nkfs_part_pitch(B, k);
	uint64_t off_ids = round16(B), off_parts = off_ids + round16((uint64_t)n);
	uint64_t in_bytes = off_parts, parts_bytes = pitch * (uint64_t)n;
	void *dv, *hv;
	if (B <= NKFS_ZC_MAX) {
		if ((err = nkfs_ctx_host(c, off_parts + parts_bytes, &hv)))
			goto out;
		uint8_t *h = hv;
		memcpy(h, block, B);
		memcpy(h + off_ids, ids, (size_t)n);
		struct nkfs_geom zg = { h, round16(B), B, NULL, NULL, h + off_parts, pitch, NULL, 1, n, k, NULL, 0, 0, NULL, 0, 0, 0, NULL };
		if ((err = nkfs_launch_encode(&zg, h + off_ids, NULL, nkfs_gf(), c->stream)) ||
		    (err = nkfs_ctx_wait(c, B >= NKFS_SPIN_MIN)))
			goto out;
		for (int i = 0; i < n; i++)
			memcpy(parts[i], h + off_parts + pitch * (uint64_t)i, ps);
		err = 0;
		goto out;
	}
	if ((err = nkfs_ctx_dev(c, off_parts + parts_bytes, &dv)) ||
	    (err = nkfs_ctx_host(c, in_bytes > parts_bytes ? in_bytes : parts_bytes, &hv)))
		goto out;
	uint8_t *d = dv, *h = hv;
	memcpy(h, block, B);
	memcpy(h + off_ids, ids, (size_t)n);
	HIPGO(hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, c->stream));
	struct nkfs_geom g = { d, round16(B), B, NULL, NULL, d + off_parts, pitch, NULL, 1, n, k, NULL, 0, 0, NULL, 0, 0, 0, NULL };
	if ((err = nkfs_launch_encode(&g, d + off_ids, NULL, nkfs_gf(), c->stream)))
		goto out;
	HIPGO(hipMemcpyAsync(h, d + off_parts, parts_bytes, hipMemcpyDeviceToHost, c->stream));
	if ((err = nkfs_ctx_wait(c, 1)))
		goto out;
	for (int i = 0; i < n; i++)
		memcpy(parts[i], h + pitch * (uint64_t)i, ps);
	err = 0;
out:
	nkfs_ctx_put(c);
	return err;
}

int nk8_split_block(uint8_t *block, uint32_t block_size, int n, int k, uint8_t ***pparts, uint8_t **pids)
{
	if (nkfs_bad_params(block_size, n, k))
		return -EINVAL;
	if (!nk8_inited || !nkfs_gpu_ready())
		return -EAGAIN;
	uint32_t ps = nkfs_part_size(block_size, k);
	uint8_t *ids = crt_malloc((size_t)n);
	uint8_t **parts = crt_malloc((size_t)n * sizeof(*parts));
	int err = -ENOMEM;
	if (!ids || !parts)
		goto fail;
	memset(parts, 0, (size_t)n * sizeof(*parts));
	for (int i = 0; i < n; i++)
		if (!(parts[i] = crt_malloc(ps)))
			goto fail;
	if ((err = gen_part_ids(ids, n)))
		goto fail;
	if ((err = gpu_split(block, block_size, n, k, ids, parts)))
		goto fail;
	*pparts = parts;
	*pids = ids;
	return 0;
fail:
	if (parts) {
		for (int i = 0; i < n; i++)
			crt_free(parts[i]);
		crt_free(parts);
	}
	crt_free(ids);
	return err;
}

int nk8_assemble_block(uint8_t **parts, uint8_t *ids, int n, int k, uint8_t *block, uint32_t block_size)
{
	if (nkfs_bad_params(block_size, n, k))
		return -EINVAL;
	if (!nk8_inited || !nkfs_gpu_ready())
		return -EAGAIN;
	/* the first k parts with distinct ids, in argument order
	 * (crt/nk8.c:512-537); only those travel to the device */
	int sel[254];
	int have = 0;
	for (int i = 0; i < n && have < k; i++) {
		int dup = 0;
		for (int j = 0; j < i; j++)
			dup |= ids[j] == ids[i];
		if (!dup)
			sel[have++] = i;
	}
	if (have < k)
		return -EINVAL;
	struct nkfs_ctx *c = nkfs_ctx_get();
	if (!c)
		return -EIO;
	int err;
	uint32_t ps = nkfs_part_size(block_size, k);
	uint64_t pitch = nkfs_part_pitch(block_size, k);
	/* device and pinned staging share one layout for the inputs:
	 * parts | ids | avail, one H2D; block | status come back in one D2H */
	uint64_t off_parts = 0;
	uint64_t off_ids = off_parts + pitch * (uint64_t)k;
	uint64_t off_avail = off_ids + 256;
	uint64_t off_work = off_avail + 256;
	uint64_t off_status = off_work + round16(nkfs_decode_work_bytes(1, k));
	uint64_t off_block = off_status + 16;
	uint64_t in_bytes = off_work, out_bytes = 16 + round16(block_size);
	void *dv, *hv;
	if (block_size <= NKFS_ZC_MAX) {
		/* zero-copy: the decode reads the parts from pinned staging and
		 * writes status and block back into it (layout as the device's) */
		if ((err = nkfs_ctx_host(c, off_block + round16(block_size), &hv)))
			goto out;
		uint8_t *h = hv;
		for (int c2 = 0; c2 < k; c2++) {
			memcpy(h + off_parts + pitch * (uint64_t)c2, parts[sel[c2]], ps);
			h[off_ids + c2] = ids[sel[c2]];
			h[off_avail + c2] = (uint8_t)c2;
		}
		struct nkfs_geom zg = { h + off_block, round16(block_size), block_size, NULL, NULL, h + off_parts, pitch,
					NULL, 1, k, k, NULL, 0, 0, NULL, 0, 0, 0, NULL };
		if ((err = nkfs_launch_decode(&zg, k, h + off_ids, h + off_avail, k, h + off_work,
					      (int32_t *)(h + off_status), nkfs_gf(), c->stream, NULL, NULL)) ||
		    (err = nkfs_ctx_wait(c, block_size >= NKFS_SPIN_MIN)))
			goto out;
		int32_t zst;
		memcpy(&zst, h + off_status, sizeof(zst));
		if (!zst)
			memcpy(block, h + off_block, block_size);
		err = zst;
		goto out;
	}
	if ((err = nkfs_ctx_dev(c, off_block + round16(block_size), &dv)) ||
	    (err = nkfs_ctx_host(c, in_bytes > out_bytes ? in_bytes : out_bytes, &hv)))
		goto out;
	uint8_t *d = dv, *h = hv;
	for (int c2 = 0; c2 < k; c2++) {
		memcpy(h + off_parts + pitch * (uint64_t)c2, parts[sel[c2]], ps);
		h[off_ids + c2] = ids[sel[c2]];
		h[off_avail + c2] = (uint8_t)c2;
	}
	HIPGO(hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, c->stream));
	struct nkfs_geom g = { d + off_block, round16(block_size), block_size, NULL, NULL, d + off_parts, pitch,
			       NULL, 1, k, k, NULL, 0, 0, NULL, 0, 0, 0, NULL };
	if ((err = nkfs_launch_decode(&g, k, d + off_ids, d + off_avail, k, d + off_work,
				      (int32_t *)(d + off_status), nkfs_gf(), c->stream, NULL, NULL)))
		goto out;
	HIPGO(hipMemcpyAsync(h, d + off_status, 16 + block_size, hipMemcpyDeviceToHost, c->stream));
	if ((err = nkfs_ctx_wait(c, 1)))
		goto out;
	int32_t st;
	memcpy(&st, h, sizeof(st));
	if (!st)
		memcpy(block, h + 16, block_size);
	err = st;
out:
	nkfs_ctx_put(c);
	return err;
}

/* The reference's load-time self test (crt/nk8.c:601-723, run 5x by
 * nk8_init :735-744): random block -> split -> k random distinct parts ->
 * assemble -> XXH64 of input and output must match.  Here every step after
 * the random draw runs on the GPU. */
static int self_test(uint32_t block_size, int n, int k)
{
	int err = -ENOMEM;
	uint8_t *block = crt_malloc(block_size), *result = crt_malloc(block_size);
	uint8_t **parts = NULL, *ids = NULL;
	uint8_t *sparts[254], sids[254];
	if (!block || !result)
		goto out;
	if ((err = rand_bytes(block, block_size)))
		goto out;
	uint64_t in_sum = XXH64(block, block_size, 0);
	if ((err = nk8_split_block(block, block_size, n, k, &parts, &ids)))
		goto out;
	for (int i = 0; i < k; i++) {
		for (;;) {
			uint32_t j;
			if ((err = rand_below((uint32_t)n, &j)))
				goto out;
			int used = 0;
			for (int m = 0; m < i; m++)
				used |= sparts[m] == parts[j];
			if (!used) {
				sparts[i] = parts[j];
				sids[i] = ids[j];
				break;
			}
		}
	}
	if ((err = nk8_assemble_block(sparts, sids, k, k, result, block_size)))
		goto out;
	err = XXH64(result, block_size, 0) == in_sum ? 0 : -EINVAL;
	if (err)
		fprintf(stderr, "nkfs: nk8 self test mismatch (block_size %u n %d k %d)\n", block_size, n, k);
out:
	if (parts) {
		for (int i = 0; i < n; i++)
			crt_free(parts[i]);
		crt_free(parts);
	}
	crt_free(ids);
	crt_free(result);
	crt_free(block);
	return err;
}

static uint32_t rand_min_max(uint32_t lo, uint32_t hi)
{
	uint32_t v = 0;
	if (lo >= hi || rand_below(hi - lo + 1, &v))
		return lo;
	return lo + v;
}

int nk8_init(void)
{
	int err = nkfs_gpu_init(-1);
	if (err)
		return err;
	nk8_inited = 1;
	for (int i = 0; i < 5; i++) {
		uint32_t size = rand_min_max(3000, 70000);
		int k = (int)rand_min_max(2, 254);
		int n = (int)rand_min_max((uint32_t)k, 255);
		if ((err = self_test(size, n, k)))
			return err;
	}
	return 0;
}

/* crt/nk8.c:749-752 is empty: the tables stay valid.  Here the idle
 * per-call contexts (streams, scratch) are returned to the driver; the
 * device tables stay, so later calls keep working as in the reference. */
void nk8_release(void)
{
	nkfs_ctx_trim();
}
