/*
 * pipeline.c -- host-memory entry points: sub-batches streamed through the
 * GPU on two streams so that PCIe H2D, the fused kernels and PCIe D2H
 * overlap (the reference's path starts and ends in host memory: client
 * socket -> core/upages.c page buffers -> block device).
 */
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "../../include/nkfs_gpu.h"
#include "nkfs_internal.h"
#include "runtime.h"

/* pin a caller buffer for the call unless the runtime already knows it */
static int pin(const void *p, size_t bytes, int *registered)
{
	*registered = 0;
	if (!p || !bytes)
		return 0;
	hipPointerAttribute_t attr;
	if (hipPointerGetAttributes(&attr, p) == hipSuccess && attr.type == hipMemoryTypeHost)
		return 0;
	(void)hipGetLastError();
	hipError_t e = hipHostRegister((void *)p, bytes, hipHostRegisterDefault);
	if (e == hipErrorHostMemoryAlreadyRegistered) {
		(void)hipGetLastError();
		return 0;
	}
	if (e != hipSuccess)
		return nkfs_hip_fail("hipHostRegister", (int)e);
	*registered = 1;
	return 0;
}

/* Three sub-batches in flight (H2D of one, kernels of another, D2H of a
 * third); each rides a pooled context (its stream and growable device
 * scratch are reused across calls, so a call creates no streams and
 * allocates no device memory once warm). */
#define NSTREAM 3

int nkfs_nk8_encode_host(const uint8_t *h_blocks, uint64_t block_pitch, uint32_t block_size, uint32_t nstripes,
			 int n, int k, const uint8_t *h_ids, uint8_t *h_parts, uint64_t part_pitch,
			 uint64_t *h_digests, uint64_t chunk_bytes)
{
	if (nkfs_bad_params(block_size, n, k))
		return -EINVAL;
	if (!nkfs_gpu_ready())
		return -EAGAIN;
	if (!nstripes)
		return 0;
	if (!h_blocks || !h_ids || !h_parts || part_pitch < nkfs_part_size(block_size, k) || (part_pitch & 15) ||
	    (nstripes > 1 && block_pitch < block_size))
		return -EINVAL;
	if (!chunk_bytes)
		chunk_bytes = 32ull << 20;
	uint32_t per = (uint32_t)(chunk_bytes / block_size);
	if (per < 1)
		per = 1;
	if (per > nstripes)
		per = nstripes;

	const uint64_t bp = block_pitch ? block_pitch : block_size;
	const uint64_t in_bytes = (uint64_t)(nstripes - 1) * bp + block_size;
	const uint64_t parts_bytes = (uint64_t)nstripes * n * part_pitch;
	int reg[4] = {0, 0, 0, 0}, err;
	struct nkfs_ctx *cx[NSTREAM] = {0};
	if ((err = pin(h_blocks, in_bytes, &reg[0])) || (err = pin(h_ids, (size_t)nstripes * n, &reg[1])) ||
	    (err = pin(h_parts, parts_bytes, &reg[2])) ||
	    (err = pin(h_digests, h_digests ? (size_t)nstripes * n * 8 : 0, &reg[3])))
		goto unpin;

	/* per context: blocks | parts | ids | digests (device) */
	const uint64_t dblk = (uint64_t)per * bp;
	const uint64_t dparts = (uint64_t)per * n * part_pitch;
	const uint64_t dids = ((uint64_t)per * n + 255) & ~255ull;
	const uint64_t ddig = (uint64_t)per * n * 8;
	const uint64_t slot = ((dblk + 255) & ~255ull) + dparts + dids + ddig;
	void *dev[NSTREAM];
	hipError_t e = hipSuccess;
	for (int i = 0; i < NSTREAM; i++) {
		cx[i] = nkfs_ctx_get();
		if (!cx[i]) {
			err = -ENOMEM;
			goto out;
		}
		if ((err = nkfs_ctx_dev(cx[i], slot, &dev[i])))
			goto out;
	}
	for (uint32_t s0 = 0, it = 0; s0 < nstripes; s0 += per, it++) {
		const uint32_t cnt = nstripes - s0 < per ? nstripes - s0 : per;
		hipStream_t s = cx[it % NSTREAM]->stream;
		uint8_t *d = (uint8_t *)dev[it % NSTREAM];
		uint8_t *d_blk = d, *d_parts = d + ((dblk + 255) & ~255ull);
		uint8_t *d_ids = d_parts + dparts;
		uint64_t *d_dig = (uint64_t *)(d_ids + dids);
		const uint64_t nin = (uint64_t)(cnt - 1) * bp + block_size;
		if ((e = hipMemcpyAsync(d_blk, h_blocks + (uint64_t)s0 * bp, nin, hipMemcpyHostToDevice, s)) ||
		    (e = hipMemcpyAsync(d_ids, h_ids + (uint64_t)s0 * n, (size_t)cnt * n, hipMemcpyHostToDevice, s))) {
			err = nkfs_hip_fail("H2D", (int)e);
			goto out;
		}
		struct nkfs_geom g = { d_blk, bp, block_size, NULL, NULL, d_parts, part_pitch, NULL, cnt, n, k, NULL, 0, 0 };
		if ((err = nkfs_launch_encode(&g, d_ids, h_digests ? d_dig : NULL, nkfs_gf(), s)))
			goto out;
		if ((e = hipMemcpyAsync(h_parts + (uint64_t)s0 * n * part_pitch, d_parts, (uint64_t)cnt * n * part_pitch,
					hipMemcpyDeviceToHost, s)) ||
		    (h_digests && (e = hipMemcpyAsync(h_digests + (uint64_t)s0 * n, d_dig, (size_t)cnt * n * 8,
						       hipMemcpyDeviceToHost, s)))) {
			err = nkfs_hip_fail("D2H", (int)e);
			goto out;
		}
	}
	err = 0;
out:
	for (int i = 0; i < NSTREAM; i++)
		if (cx[i]) {
			if ((e = hipStreamSynchronize(cx[i]->stream)) != hipSuccess && !err)
				err = nkfs_hip_fail("pipeline sync", (int)e);
			nkfs_ctx_put(cx[i]);
		}
unpin:
	if (reg[0])
		hipHostUnregister((void *)h_blocks);
	if (reg[1])
		hipHostUnregister((void *)h_ids);
	if (reg[2])
		hipHostUnregister(h_parts);
	if (reg[3])
		hipHostUnregister(h_digests);
	return err;
}

/* Ragged host batch: stripe s is h_block_size[s] bytes at h_blocks +
 * h_block_off[s]; its n parts go to h_parts + h_part_off[s] + i*pitch(B_s).
 * Offsets must be non-decreasing in s (a packed layout), so a run of
 * consecutive stripes is one contiguous byte range on both sides: each
 * sub-batch is one H2D of its blocks, one launch of the ragged encode and one
 * D2H of its parts.  The device geometry points its bases at (device buffer -
 * first offset), so the caller's offsets are copied unchanged. */
int nkfs_nk8_encode_ragged_host(const uint8_t *h_blocks, const uint64_t *h_block_off, const uint32_t *h_block_size,
				uint32_t max_block_size, uint32_t nstripes, int n, int k, const uint8_t *h_ids,
				uint8_t *h_parts, const uint64_t *h_part_off, uint64_t *h_digests, uint64_t chunk_bytes)
{
	if (nkfs_bad_params(max_block_size, n, k))
		return -EINVAL;
	if (!nkfs_gpu_ready())
		return -EAGAIN;
	if (!nstripes)
		return 0;
	if (!h_blocks || !h_block_off || !h_block_size || !h_ids || !h_parts || !h_part_off)
		return -EINVAL;
	if (!chunk_bytes)
		chunk_bytes = 32ull << 20;

	/* sub-batches: [first stripe, end) with <= chunk_bytes of blocks (>= 1
	 * stripe); byte extents of every range on both sides */
	uint64_t in_end = 0, parts_end = 0, max_in = 0, max_parts = 0, max_cnt = 0;
	for (uint32_t s = 0; s < nstripes; s++) {
		if (h_block_size[s] > max_block_size || (s && (h_block_off[s] < h_block_off[s - 1] ||
							     h_part_off[s] < h_part_off[s - 1])))
			return -EINVAL;
		const uint64_t e1 = h_block_off[s] + h_block_size[s];
		const uint64_t e2 = h_part_off[s] + (uint64_t)n * nkfs_part_pitch(h_block_size[s], k);
		in_end = e1 > in_end ? e1 : in_end;
		parts_end = e2 > parts_end ? e2 : parts_end;
	}
	for (uint32_t s0 = 0; s0 < nstripes;) {
		uint32_t s1 = s0 + 1;
		uint64_t hi = h_block_off[s0] + h_block_size[s0];
		while (s1 < nstripes && h_block_off[s1] + h_block_size[s1] - h_block_off[s0] <= chunk_bytes) {
			const uint64_t e = h_block_off[s1] + h_block_size[s1];
			hi = e > hi ? e : hi;
			s1++;
		}
		uint64_t phi = 0;
		for (uint32_t s = s0; s < s1; s++) {
			const uint64_t e = h_part_off[s] + (uint64_t)n * nkfs_part_pitch(h_block_size[s], k);
			phi = e > phi ? e : phi;
		}
		if (hi - h_block_off[s0] > max_in)
			max_in = hi - h_block_off[s0];
		if (phi - h_part_off[s0] > max_parts)
			max_parts = phi - h_part_off[s0];
		if (s1 - s0 > max_cnt)
			max_cnt = s1 - s0;
		s0 = s1;
	}

	int reg[7] = {0, 0, 0, 0, 0, 0, 0}, err;
	struct nkfs_ctx *cx[NSTREAM] = {0};
	if ((err = pin(h_blocks, in_end, &reg[0])) || (err = pin(h_ids, (size_t)nstripes * n, &reg[1])) ||
	    (err = pin(h_parts, parts_end, &reg[2])) ||
	    (err = pin(h_digests, h_digests ? (size_t)nstripes * n * 8 : 0, &reg[3])) ||
	    (err = pin(h_block_off, (size_t)nstripes * 8, &reg[4])) ||
	    (err = pin(h_block_size, (size_t)nstripes * 4, &reg[5])) ||
	    (err = pin(h_part_off, (size_t)nstripes * 8, &reg[6])))
		goto unpin;

	/* per context: blocks | parts | block_off | part_off | sizes | ids | digests */
	const uint64_t a_in = (max_in + 255) & ~255ull, a_parts = (max_parts + 255) & ~255ull;
	const uint64_t a_off = (max_cnt * 8 + 255) & ~255ull, a_sz = (max_cnt * 4 + 255) & ~255ull;
	const uint64_t a_ids = (max_cnt * n + 255) & ~255ull, a_dig = max_cnt * n * 8;
	const uint64_t slot = a_in + a_parts + 2 * a_off + a_sz + a_ids + a_dig;
	void *dev[NSTREAM];
	hipError_t e = hipSuccess;
	for (int i = 0; i < NSTREAM; i++) {
		cx[i] = nkfs_ctx_get();
		if (!cx[i]) {
			err = -ENOMEM;
			goto out;
		}
		if ((err = nkfs_ctx_dev(cx[i], slot, &dev[i])))
			goto out;
	}
	for (uint32_t s0 = 0, it = 0; s0 < nstripes; it++) {
		uint32_t s1 = s0 + 1;
		uint64_t hi = h_block_off[s0] + h_block_size[s0];
		while (s1 < nstripes && h_block_off[s1] + h_block_size[s1] - h_block_off[s0] <= chunk_bytes) {
			const uint64_t e1 = h_block_off[s1] + h_block_size[s1];
			hi = e1 > hi ? e1 : hi;
			s1++;
		}
		uint64_t phi = 0;
		for (uint32_t s = s0; s < s1; s++) {
			const uint64_t e2 = h_part_off[s] + (uint64_t)n * nkfs_part_pitch(h_block_size[s], k);
			phi = e2 > phi ? e2 : phi;
		}
		const uint32_t cnt = s1 - s0;
		const uint64_t lo = h_block_off[s0], plo = h_part_off[s0];
		hipStream_t st = cx[it % NSTREAM]->stream;
		uint8_t *d = (uint8_t *)dev[it % NSTREAM];
		uint8_t *d_blk = d, *d_parts = d + a_in;
		uint64_t *d_boff = (uint64_t *)(d_parts + a_parts), *d_poff = (uint64_t *)((uint8_t *)d_boff + a_off);
		uint32_t *d_sz = (uint32_t *)((uint8_t *)d_poff + a_off);
		uint8_t *d_ids = (uint8_t *)d_sz + a_sz;
		uint64_t *d_dig = (uint64_t *)(d_ids + a_ids);
		if ((e = hipMemcpyAsync(d_blk, h_blocks + lo, hi - lo, hipMemcpyHostToDevice, st)) ||
		    (e = hipMemcpyAsync(d_boff, h_block_off + s0, (size_t)cnt * 8, hipMemcpyHostToDevice, st)) ||
		    (e = hipMemcpyAsync(d_poff, h_part_off + s0, (size_t)cnt * 8, hipMemcpyHostToDevice, st)) ||
		    (e = hipMemcpyAsync(d_sz, h_block_size + s0, (size_t)cnt * 4, hipMemcpyHostToDevice, st)) ||
		    (e = hipMemcpyAsync(d_ids, h_ids + (uint64_t)s0 * n, (size_t)cnt * n, hipMemcpyHostToDevice, st))) {
			err = nkfs_hip_fail("H2D", (int)e);
			goto out;
		}
		/* bases shifted by the range's first offsets: base + off[s] lands
		 * inside this context's buffers */
		struct nkfs_geom g = { d_blk - lo, 0, max_block_size, d_boff, d_sz, d_parts - plo, 0, d_poff, cnt, n, k,
				       NULL, 0, 0 };
		if ((err = nkfs_launch_encode(&g, d_ids, h_digests ? d_dig : NULL, nkfs_gf(), st)))
			goto out;
		if ((e = hipMemcpyAsync(h_parts + plo, d_parts, phi - plo, hipMemcpyDeviceToHost, st)) ||
		    (h_digests && (e = hipMemcpyAsync(h_digests + (uint64_t)s0 * n, d_dig, (size_t)cnt * n * 8,
						       hipMemcpyDeviceToHost, st)))) {
			err = nkfs_hip_fail("D2H", (int)e);
			goto out;
		}
		s0 = s1;
	}
	err = 0;
out:
	for (int i = 0; i < NSTREAM; i++)
		if (cx[i]) {
			if ((e = hipStreamSynchronize(cx[i]->stream)) != hipSuccess && !err)
				err = nkfs_hip_fail("pipeline sync", (int)e);
			nkfs_ctx_put(cx[i]);
		}
unpin:
	if (reg[0])
		hipHostUnregister((void *)h_blocks);
	if (reg[1])
		hipHostUnregister((void *)h_ids);
	if (reg[2])
		hipHostUnregister(h_parts);
	if (reg[3])
		hipHostUnregister(h_digests);
	if (reg[4])
		hipHostUnregister((void *)h_block_off);
	if (reg[5])
		hipHostUnregister((void *)h_block_size);
	if (reg[6])
		hipHostUnregister((void *)h_part_off);
	return err;
}
