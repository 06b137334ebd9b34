/* nkfs_internal.h -- contract between the C host side (nk8.c, csum.c,
 * runtime.c) and the HIP launchers (nk8_kernels.hip).  Plain C types only. */
#ifndef NKFS_INTERNAL_H
#define NKFS_INTERNAL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Geometry of a batch of stripes in device memory.  Uniform batches set
 * block_sizes == NULL and use (block_pitch, block_size, part_pitch); ragged
 * batches give per-stripe block offsets/sizes and part offsets, with the
 * part pitch of stripe s fixed at nkfs_part_pitch(block_sizes[s], k). */
struct nkfs_geom {
	const uint8_t *blocks;
	uint64_t block_pitch;
	uint32_t block_size;
	const uint64_t *block_off;
	const uint32_t *block_sizes;
	uint8_t *parts;
	uint64_t part_pitch;
	const uint64_t *part_off;
	uint32_t nstripes;
	int n;
	int k;
	/* optional processing order (ragged batches): wave slot i handles stripe
	 * order[i]; NULL = identity.  Only changes which stripes share a wave and
	 * when they run, never an output. */
	const uint32_t *order;
	/* optional part-size window (fast encoders only): a launch processes
	 * only the stripes whose part size lies in [part_min, part_max), 0 =
	 * unbounded.  Two launches with complementary windows split one ragged
	 * batch between two kernels. */
	uint32_t part_min;
	uint32_t part_max;
	/* optional device scratch for a launch's own metadata (the ragged
	 * size order, the ragged slice map): the host pipeline carves it from
	 * its context buffer; NULL = stream-ordered scratch from the library's
	 * private memory pool (nkfs_scratch_alloc). */
	uint8_t *scratch;
	uint64_t scratch_bytes;
	/* optional bounds of the caller's block / part buffers (bytes from
	 * `blocks` / `parts`), checked by the debug-bounds build's device
	 * asserts (make DEBUG_BOUNDS=1); 0 = unknown. */
	uint64_t blocks_bytes;
	uint64_t parts_bytes;
	/* optional zeroed device word: the group counter of a persistent launch
	 * over g.order (k_order_by_size zeroes it; with_size_order sets it) */
	uint32_t *queue;
};

/* Scratch bytes the launchers take from nkfs_geom.scratch for a ragged
 * batch of `nstripes` stripes whose parts span `sum_units` 1,024-row units
 * in all (sum over stripes of ceil(part_size / 1024)). */
uint64_t nkfs_ragged_scratch_bytes(uint32_t nstripes, uint64_t sum_units);

/* Hash waves per warp-specialised workgroup (n > 4) for a batch of s
 * stripes: one CU holds one workgroup, so a grid that ends in a partial
 * round of workgroups wastes CUs.  Two hash waves (four stripes per
 * workgroup) whenever their rounds, at twice the work each, take no longer
 * than one hash wave's: 768 / 1,024 / 8,192 stripes -> 2; 384 / 512 /
 * 1,536 -> 1 (profiles/r04/seam_mid.txt, seam_sweep_r04_boxA.txt). */
static inline int nkfs_ws_auto_hash_waves(uint32_t s)
{
	return 2ull * (((uint64_t)s + 1023u) / 1024u) <= ((uint64_t)s + 511u) / 512u ? 2 : 1;
}

/* Kernel choice and launch shape (struct nkfs_tune, include/nkfs_gpu.h):
 * one process-wide copy, set at init, read by the launchers. */
struct nkfs_tune;

/* Launchers: return 0 or a negative errno; `stream` is a hipStream_t. */
int nkfs_launch_gf_init(void *gf_tables, void *stream);
int nkfs_launch_encode(const struct nkfs_geom *g, const uint8_t *ids,
		       uint64_t *digests, const void *gf_tables, void *stream);
int nkfs_launch_hash_parts(const struct nkfs_geom *g, uint64_t *digests,
			   void *stream);
int nkfs_launch_decode(const struct nkfs_geom *g, int n_slots,
		       const uint8_t *ids, const uint8_t *avail, int navail,
		       void *work, int32_t *status, const void *gf_tables,
		       void *stream, const uint64_t *expect, uint64_t *badmask);
/* One message's XXH64 chains in one wave (xxh64_chain.hip): fold `nst`
 * 32-byte stripes at `src` (a device-visible pointer: pinned host memory or
 * device memory) into the accumulators -- from v[] or, with FROM_DEV, from
 * v_dev[] -- then with TO_DEV store them to v_dev[], with EMIT store them
 * to out[2..5], with FINISH merge, add total_len, fold the tail (tail_len <
 * 32 bytes, by value), avalanche and store out[0] = digest; after EMIT or
 * FINISH out[1] = flag (system-scope release: the host spins on it). */
enum { NKFS_XXH_FROM_DEV = 1, NKFS_XXH_TO_DEV = 2, NKFS_XXH_FINISH = 4, NKFS_XXH_EMIT = 8 };
struct nkfs_xxh_args {
	uint64_t v[4];
	uint64_t total_len;
	uint64_t seed;
	uint64_t nst;
	const uint8_t *src;
	uint64_t *v_dev;
	uint64_t *out;
	uint64_t flag;
	uint8_t tail[32];
	uint32_t tail_len;
	uint32_t flags;
};
int nkfs_launch_xxh64_chain(const struct nkfs_xxh_args *a, void *stream);
/* Mailbox of the per-call service wave (k_xxh64_service): the host writes
 * op and args, then seq (release) into the request box (coherent host
 * memory, or device memory through the BAR); the wave copies the args,
 * stores taken = seq into the answer box (host memory), runs the message
 * and stores its completion word; alive (answer box) drops to 0 when the
 * wave leaves. */
#define NKFS_SVC_XXH 1u
#define NKFS_SVC_STOP 2u
#define NKFS_SVC_XXH_INL 3u  /* the message's stripes (<= 1 KiB) are in inl */
#define NKFS_SVC_INL 1024u
struct nkfs_svc_box {
	uint64_t seq;
	uint64_t op;
	struct nkfs_xxh_args args;
	uint64_t taken;
	uint64_t alive;
	uint8_t inl[NKFS_SVC_INL] __attribute__((aligned(64)));
};
int nkfs_launch_xxh64_service(struct nkfs_svc_box *mb, struct nkfs_svc_box *ob, uint64_t idle_ticks,
			      uint64_t life_ticks, void *stream);
int nkfs_launch_xxh64_batch(const uint8_t *base, const uint64_t *off,
			    const uint64_t *len, uint32_t count, uint64_t seed,
			    uint64_t *out, void *stream);
int nkfs_fast_xxh64_strided(const uint8_t *base, uint64_t pitch,
			    uint64_t len, uint32_t count, uint64_t *out,
			    const uint64_t *expect, int32_t *status,
			    void *stream);
int nkfs_fast_xxh64_pages(const uint8_t *const *pages, const uint64_t *first,
			  const uint64_t *len, uint32_t count,
			  uint32_t page_shift, uint64_t *out, void *stream);
int nkfs_launch_synth(uint8_t *blocks, uint64_t block_pitch,
		      uint32_t block_size, uint32_t nstripes,
		      uint64_t seed, uint64_t first_stripe, void *stream);
int nkfs_launch_synth_ragged(uint8_t *blocks, const uint64_t *block_off, const uint32_t *block_size,
			     uint32_t nstripes, uint64_t seed, uint64_t first_stripe, void *stream);

/* Part pitch used when the library lays parts out itself (ragged batches,
 * the drop-in entry points): part_size rounded up to whole 256-byte spans so
 * that every chunk a kernel writes covers full 128-byte cache lines. */
#define NKFS_PART_ALIGN 256u

/* Compute units of the library's device (persistent grids). */
int nkfs_cu_count(void);

/* Sizes shared by host and launchers. */
uint64_t nkfs_decode_work_bytes(uint32_t nstripes, int k);
size_t nkfs_gf_tables_bytes(void);

#ifdef __cplusplus
}
#endif
#ifdef __cplusplus
#include "../../include/nkfs_gpu.h"
/* One consistent copy of the process-wide struct nkfs_tune: nkfs_tune_get
 * copies it under its lock, so a concurrent nkfs_tune_set never tears a
 * launch's read (the launchers take one copy per decision). */
static inline nkfs_tune nkfs_tune_now()
{
	nkfs_tune t;
	nkfs_tune_get(&t);
	return t;
}
#endif

#endif
