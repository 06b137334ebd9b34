/*
 * nkfs_gpu.h -- batched, device-resident entry points of libnkfs_crt.so.
 *
 * The reference encodes one block per call with ids it draws itself
 * (crt/nk8.c:344-444) and decodes one block per call (crt/nk8.c:446-599).
 * On MI355X the same arithmetic runs over whole batches of independent
 * stripes already resident in HBM, with the ids passed in explicitly so a
 * batch is reproducible bit for bit.  All pointers named d_* are device
 * pointers; `stream` is a hipStream_t (NULL = the default stream); calls are
 * asynchronous on that stream and return 0 or a negative errno for argument
 * errors (-EINVAL), calls before nk8_init/nkfs_gpu_init (-EAGAIN) and launch
 * failures (-EIO).  No host synchronisation happens inside, so calls can be
 * captured in a hipGraph.
 *
 * Layout (uniform batch of `nstripes` stripes):
 *   block s        d_blocks + s*block_pitch, block_size bytes, interleaved
 *                  (row j = bytes j*k .. j*k+k-1, crt/nk8.c:411)
 *   part i of s    d_parts + (s*n + i)*part_pitch, part_size bytes (planar)
 *   ids of s       d_ids + s*n, n bytes (evaluation point of part i)
 *   digest (s,i)   d_digests[s*n + i] = XXH64(part, part_size, 0)
 * part_pitch must be >= nkfs_part_size(block_size, k) and a multiple of 16.
 */
#ifndef NKFS_GPU_H
#define NKFS_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Initialise the GPU side without the reference's self test (nk8_init runs
 * this plus the test).  device < 0: env NKFS_DEVICE or the current device.
 * That device is the library's device: the compatibility entry points
 * (nkfs_crt.h) run there. */
int nkfs_gpu_init(int device);
/* 1 when the library has a usable GPU context. */
int nkfs_gpu_ready(void);
/* The library's device (-1 before init) and the number of visible devices. */
int nkfs_gpu_device(void);
int nkfs_gpu_count(void);

/* Multi-GPU (stripes are independent).  Batched device
 * calls run on the device of the stream they are given (each device's
 * tables are set up on first use).  The host-memory entry points below
 * split every batch into byte-balanced contiguous stripe ranges over the
 * device lanes set here -- one host thread and three streams per lane, no
 * data exchanged between lanes; an entry may repeat (two lanes on one
 * device).  count 0 = the library's device only (the default).  Returns
 * -ENODEV for a device that does not exist. */
int nkfs_gpu_set_devices(const int *devices, int count);
/* Current lanes into devices[0..max); returns their number. */
int nkfs_gpu_get_devices(int *devices, int max);

/* Kernel choice and launch shape of the batched entry points.  The library
 * starts with the measured defaults; tools and tests replace
 * them with nkfs_tune_set to compare kernels in one process.  The launchers
 * read only this struct: no environment variable changes what runs. */
/* NKFS_ENC_WIDE: part-group encoder + a second XXH64 pass (any n, k <= 16;
 * the default beyond the fused kernels' n <= 8, k <= 8 for batches too small
 * to fill the chip); NKFS_ENC_WIDE_WS: part-group encoder with XXH64 fused
 * (a hash wave per workgroup; the default for k <= 16 batches that fill the
 * chip); NKFS_ENC_GENERIC: thread-per-row kernel; NKFS_ENC_BIG:
 * column-chunked encoder (any k; the default for k > 32, and for 16 < k <= 32
 * without digests -- with digests the stage-free encoder, tune enc_bign) */
/* NKFS_ENC_WSP: persistent warp-specialised encoder (n <= 8, k <= 8, with
 * digests; ragged batches in size order from a device-wide group counter) */
enum { NKFS_ENC_AUTO = 0, NKFS_ENC_WALK, NKFS_ENC_FUSED, NKFS_ENC_WS, NKFS_ENC_GENERIC, NKFS_ENC_WIDE, NKFS_ENC_BIG,
       NKFS_ENC_WIDE_WS, NKFS_ENC_WSP };
/* NKFS_DEC_WIDE: survivor-table decoder (k <= 16; the default for 8 < k <= 16);
 * NKFS_DEC_BIG: column-chunked decoder (any k; the default for k > 16 where
 * the stage-free decoder does not apply, tune dec_bign);
 * NKFS_DEC_RUN: run decoder (k <= 8: persistent waves, each walking one
 * contiguous run of 1,024-row units across stripes) */
/* NKFS_DEC_PAIR: k = 2 decoder (closed-form 2 x 2 inverse, one lookup per row) */
enum { NKFS_DEC_AUTO = 0, NKFS_DEC_SLICE, NKFS_DEC_WAVE, NKFS_DEC_GENERIC, NKFS_DEC_WIDE, NKFS_DEC_BIG, NKFS_DEC_RUN,
       NKFS_DEC_PAIR };
struct nkfs_tune {
	int enc_kernel;       /* NKFS_ENC_*: encoder (WIDE / GENERIC also pin n <= 8 shapes) */
	int dec_kernel;       /* NKFS_DEC_*: decoder (WIDE / GENERIC also pin k <= 8) */
	int enc_waves_per_cu; /* resident waves per CU of the walk encoder (1..32) */
	int dec_waves_per_cu; /* resident waves per CU of the slice decoder (1..32) */
	int dec_units;        /* 1,024-row units per slice-decoder wave (1, 2 or 4) */
	int enc_nib;          /* walk encoder, n > 4: nibble product tables (-1 auto, 0, 1) */
	int enc_units;        /* walk encoder: 1,024-row units per chunk (0 auto, 1, 2; n <= 4 only) */
	int size_order;       /* ragged batches run largest stripe first (0/1) */
	int enc_prefetch;     /* walk encoder: chunks of loads in flight ahead of the one encoded (1, 2) */
	int enc_fused_waves_per_cu; /* fused encoder: resident waves per CU cap (0 = none, 3..32) */
	int dec_wave_waves_per_cu;  /* wave-per-stripe decoder: same cap */
	int dec_run_units;    /* run decoder: 1,024-row units per chunk (1, 2, 4, 8, 16) */
	int enc_ws_prefetch;  /* warp-specialised encoders (n > 4, and the n > 8 fused part-group encoder): chunks of
	                         loads in flight per encoder wave (1, 2; default 2) */
	int enc_big_fused;    /* column-chunked k > 16 encoder: 1 = XXH64 fused (traffic 1.0x), 0 = second pass, -1 = auto
	                         (default: the second pass -- W3 +10 % with the diagonal tables; 16 < k <= 32 with digests
	                         take the stage-free encoder) */
	int dec_pair_stage;   /* k = 2 decoder: 1 = output through an LDS stage (1 KiB runs per store), 0 = direct */
	int host_depth;       /* host-memory entry points: sub-batches in flight per lane (2..8) */
	int host_lanes;       /* host-memory entry points: host threads (lanes) per device (1..4) */
	int enc_ragged_split; /* ragged n > 4 encode: parts >= this many bytes on the warp-specialised kernel (0 = all walk) */
	int enc_ws_waves;     /* warp-specialised encoder, n > 4: encoder waves per workgroup (4 default, or 6) */
	int dec_pair_waves;   /* k = 2 decoder: waves (one stripe each) per workgroup (1 or 4) */
	int enc_few_max;      /* n <= 8 encode of at most this many big stripes (< 16 MiB of parts): the row-parallel
	                         general kernels + a hash pass instead of one wave per stripe (0..63) */
	int enc_ws_hash_waves; /* warp-specialised encoder, n > 4 with 4 encoder waves: hash waves per workgroup
	                          (0 auto: 2 from 1,024 stripes on; 1; 2) */
	int enc_persist;      /* n > 4 with digests: the persistent warp-specialised encoder (NKFS_ENC_WSP) where the
	                         automatic choice is the walk encoder (ragged batches: 1, the default) or also the
	                         warp-specialised grid (uniform batches: 2); 0 = off */
	int dec_bign;         /* k > 8 decode on the stage-free decoder (nk8_bign.hip): -2 = auto (NKFS_DEC_AUTO only:
	                         diagonal byte tables (4) for k % 4 == 0 except 16, layout 5 for the other 16 < k <= 64),
	                         -1 = off (survivor-table / column-chunked
	                         decoders), 0 = byte tables, 1 = nibble tables x 16 replicas (every
	                         lookup in its lane's own bank slot) in 16-survivor chunks, 2 = the same in 8-survivor
	                         chunks (two workgroups per CU), 3 = every output column of a slice in one workgroup
                         (8 < k <= 64; rows through an LDS stage, so odd k store whole 16-byte pieces),
	                         4 = byte tables in the diagonal layout (entry x of survivor j at x * 256 + j * 16, lane l
	                         walking the survivors from l & 15: every lookup of a lane group in its own bank slot),
	                         5 = layout 3 with diagonal tables (k <= 48; beyond, layout 3) */
	int enc_bign;         /* k <= 76 encode on the stage-free encoder with a hash wave (nk8_bign.hip; units of 16
	                         parts up to k = 32, of 8 parts above): -1 = auto
	                         (16 < k <= 32 with digests, persistent), 0 = off (column-chunked encoder + XXH64
	                         pass), 1 = every k <= 76 batch it accepts, persistent (a workgroup per CU walking
	                         the (stripe, part group) units), 2 = the same, one workgroup per unit, 3 = persistent
	                         with diagonal (bank-conflict-free) tables for every 16 < k <= 32 (automatic for
	                         k = 32) */
	int dec_pair_pipe;    /* k = 2 decode of uniform batches of blocks <= 4 KiB (C2): waves per CU of the persistent
	                         pipelined pair decoder (next stripes' slots, ids and parts in flight under the current
	                         one), taken automatically when > 0; 0 = the wave decoder */
};
void nkfs_tune_get(struct nkfs_tune *t);    /* copies under a lock: thread-safe */
int nkfs_tune_set(const struct nkfs_tune *t); /* -EINVAL on out-of-range fields; thread-safe */
/* 1 when every buffer offset the walk encoder forms for this shape fits 31
 * bits (block bytes + a chunk's reach, a stripe's part span, the digest
 * array), else 0: the launcher then takes the general kernels. */
int nkfs_walk_offsets_fit(uint64_t block_size, uint64_t part_span, uint64_t nstripes, uint64_t n);
/* CPU-only replay of the plan a ragged host call (nkfs_nk8_encode_ragged_host
 * / _decode_ragged_host, or the page-list forms when page_size > 0) makes:
 * sub-batch cuts, device layout, shifted offsets; checks that every kernel
 * access and copy of every sub-batch stays inside its region.  0 (msg: a
 * summary), -ERANGE (msg: the first violation) or -EINVAL.  No GPU call. */
int nkfs_pipeline_check(int decode, const uint64_t *block_off, const uint32_t *block_size, uint32_t max_block_size,
			uint32_t nstripes, int n_slots, int k, int navail, const uint64_t *part_off, uint32_t page_size,
			uint64_t chunk_bytes, char *msg, size_t msg_len);
/* The device of every host lane a host-memory call runs (CPU only, no GPU
 * call): struct nkfs_tune.host_lanes lanes per device, interleaved over the
 * devices (d0, d1, ..., d0, d1, ...) so a cap of max_lanes drops whole
 * rounds, never a device.  Returns the number of lanes written. */
int nkfs_host_lane_plan(const int *devices, int ndev, int per_device, int *lanes, int max_lanes);
/* Opt-in per-call service (0 off, the default; 1 on, mailbox in coherent
 * host memory; 2 on, the request half of the mailbox in device memory the
 * host writes through the PCIe BAR -- needs a host-mapped device aperture):
 * one wave stays resident on the calling thread's device and polls the
 * mailbox, so a per-call XXH64 / csum digest of a message up to 256 KiB
 * (XXH64(), csum_digest, XXH64_digest without an earlier 256 KiB fold)
 * needs no kernel launch.  The wave leaves after 20 ms without requests and
 * is relaunched by the next one; requests are serialised.  0, -EINVAL,
 * -ENODEV, -ENOMEM or -EIO. */
int nkfs_percall_service(int on);

/* ceil(block_size/k) -- crt/nk8.c:311-317. */
uint32_t nkfs_part_size(uint32_t block_size, int k);
/* part_size rounded up to 256 bytes: the pitch ragged batches and the
 * drop-in entry points use, and the recommended pitch for uniform batches
 * (every chunk the encoder writes then covers whole cache lines). */
uint64_t nkfs_part_pitch(uint32_t block_size, int k);

/* Encode (+ XXH64 of every part when d_digests != NULL) a uniform batch.
 * Same parameter rules as nk8_split_block; ids must be nonzero. */
int nkfs_nk8_encode(const uint8_t *d_blocks, uint64_t block_pitch,
		    uint32_t block_size, uint32_t nstripes, int n, int k,
		    const uint8_t *d_ids, uint8_t *d_parts, uint64_t part_pitch,
		    uint64_t *d_digests, void *stream);

/* Ragged batch (stripes of different sizes): block s at
 * d_blocks + d_block_off[s] with d_block_size[s] bytes; part i of s at
 * d_parts + d_part_off[s] + i*nkfs_part_pitch(d_block_size[s], k).
 * max_block_size bounds every d_block_size[s]. */
int nkfs_nk8_encode_ragged(const uint8_t *d_blocks, const uint64_t *d_block_off,
			   const uint32_t *d_block_size, uint32_t max_block_size,
			   uint32_t nstripes, int n, int k, const uint8_t *d_ids,
			   uint8_t *d_parts, const uint64_t *d_part_off,
			   uint64_t *d_digests, void *stream);

/* Decode a uniform batch.  Parts live in slots laid out as the encoder's
 * output (n_slots per stripe, pitch part_pitch); d_ids[s*n_slots + j] is the
 * id of slot j.  d_avail[s*navail + c] lists the slots offered for stripe s
 * in caller order; like nk8_assemble_block the first k with distinct ids
 * are used.  Every d_avail entry must be below n_slots (the host-memory
 * forms check h_avail and return -EINVAL).  d_work: nkfs_decode_workspace(nstripes, k) bytes of device
 * scratch.  d_status[s] (may be NULL) receives 0 or -EINVAL (fewer than k
 * distinct ids) per stripe; such stripes are left unwritten. */
uint64_t nkfs_decode_workspace(uint32_t nstripes, int k);
int nkfs_nk8_decode(const uint8_t *d_parts, uint64_t part_pitch, int n_slots,
		    const uint8_t *d_ids, const uint8_t *d_avail, int navail,
		    int k, uint32_t block_size, uint8_t *d_blocks,
		    uint64_t block_pitch, uint32_t nstripes, void *d_work,
		    int32_t *d_status, void *stream);

/* Ragged decode: the layout nkfs_nk8_encode_ragged writes.  Stripe s has
 * n_slots part slots at d_parts + d_part_off[s] + j*nkfs_part_pitch(
 * d_block_size[s], k) (d_part_off[s] a multiple of 16) and is rebuilt into
 * d_blocks + d_block_off[s], d_block_size[s] bytes; max_block_size bounds
 * every d_block_size[s].  Selection, status and workspace as
 * nkfs_nk8_decode (crt/nk8.c:446-599 per stripe). */
int nkfs_nk8_decode_ragged(const uint8_t *d_parts, const uint64_t *d_part_off,
			   int n_slots, const uint8_t *d_ids,
			   const uint8_t *d_avail, int navail, int k,
			   uint8_t *d_blocks, const uint64_t *d_block_off,
			   const uint32_t *d_block_size,
			   uint32_t max_block_size, uint32_t nstripes,
			   void *d_work, int32_t *d_status, void *stream);

/* nkfs_nk8_decode that also verifies every part it reads against its stored
 * digest (d_expect[s*n_slots + j] = XXH64 of slot j, as produced by
 * nkfs_nk8_encode), the GET-side check of the core's per-block sums
 * (core/inode.c:561-575).  The check is fused into the rebuild (no second
 * pass over the parts).  A stripe with a mismatching part gets status -EIO
 * and d_badmask[s] (may be NULL) bit j set for each failing slot j < 63
 * (bit 63 for slots >= 63); the rebuilt block is still written. */
int nkfs_nk8_decode_verify(const uint8_t *d_parts, uint64_t part_pitch,
			   int n_slots, const uint8_t *d_ids,
			   const uint8_t *d_avail, int navail, int k,
			   uint32_t block_size, uint8_t *d_blocks,
			   uint64_t block_pitch, uint32_t nstripes,
			   void *d_work, int32_t *d_status,
			   const uint64_t *d_expect, uint64_t *d_badmask,
			   void *stream);

/* nkfs_nk8_decode_ragged with the part check of nkfs_nk8_decode_verify
 * (d_expect[s*n_slots + j] = XXH64 of slot j; status -EIO + d_badmask). */
int nkfs_nk8_decode_ragged_verify(const uint8_t *d_parts, const uint64_t *d_part_off, int n_slots,
				  const uint8_t *d_ids, const uint8_t *d_avail, int navail, int k,
				  uint8_t *d_blocks, const uint64_t *d_block_off,
				  const uint32_t *d_block_size, uint32_t max_block_size,
				  uint32_t nstripes, void *d_work, int32_t *d_status,
				  const uint64_t *d_expect, uint64_t *d_badmask, void *stream);

/* XXH64 of `count` messages d_base + d_off[i], d_len[i] bytes each
 * (d_off[i] a multiple of 8) -- the batched form of csum_* for the core's
 * per-64 KiB-block integrity sums (core/dio.c:26-37). */
int nkfs_xxh64_batch(const uint8_t *d_base, const uint64_t *d_off,
		     const uint64_t *d_len, uint32_t count, uint64_t seed,
		     uint64_t *d_out, void *stream);

/* The core's per-cluster integrity sum, batched:
 * d_sums[i] = XXH64 of the whole cluster d_clusters + i*cluster_pitch,
 * cluster_size bytes, seed 0 -- dio_clu_sum / dio_pages_sum
 * (core/dio.c:26-37,844-847), which hash every page of a 64 KiB cluster
 * whatever part of it holds data.  With d_expect != NULL the compare of
 * nkfs_inode_block_check_sum (core/inode.c:561-575) is fused in:
 * d_status[i] = 0 when the sum matches d_expect[i], else -EINVAL.
 * d_clusters and cluster_pitch must be multiples of 8. */
int nkfs_clu_sum_batch(const uint8_t *d_clusters, uint64_t cluster_pitch,
		       uint32_t cluster_size, uint32_t count,
		       uint64_t *d_sums, const uint64_t *d_expect,
		       int32_t *d_status, void *stream);

/* nkfs_pages_dsum (core/upages.c:124-148), batched over page lists: payload
 * i is the first d_len[i] bytes of the pages d_pages[d_first_page[i]],
 * d_pages[d_first_page[i] + 1], ... (each page_size bytes, 8-byte aligned;
 * the reference's pages are 4 KiB), hashed as one message -> d_dsums[i].
 * The caller guarantees the page list covers d_len[i] (the reference's
 * -EINVAL/BUG_ON checks, :131-139).  page_size: power of two >= 512. */
int nkfs_pages_dsum_batch(const uint8_t *const *d_pages,
			  const uint64_t *d_first_page, const uint64_t *d_len,
			  uint32_t count, uint32_t page_size,
			  uint64_t *d_dsums, void *stream);

/* ---- host-memory entry points ----
 * The path's real ends: PUT = socket -> core/upages.c page buffers ->
 * device -> parts; GET = parts -> device -> page buffers.  Every call is
 * synchronous (returns when the outputs are in host memory) and cuts the
 * batch into sub-batches of about `chunk_bytes` of blocks (0 = 32 MiB) that
 * flow through three streams per device lane, so H2D, kernels and D2H of
 * consecutive sub-batches overlap.  Contiguous host buffers are DMA'd
 * directly when they are pinned allocations (hipHostMalloc, torch
 * pin_memory) or lie inside an nkfs_host_register range; any other buffer
 * (pageable memory, memory registered with hipHostRegister outside this
 * library, a range straddling a registration) is staged through pinned
 * scratch by host copies, as page lists are gathered into / scattered
 * from it.  Nothing is registered for a call.  Only defined outputs are written:
 * part bytes between a part's size and its pitch are unspecified, bytes
 * between stripes and the blocks of stripes that fail to decode
 * (-EINVAL: fewer than k distinct ids) keep the caller's contents.
 * A call that fails
 * publishes no status, digests or decoded pages of the sub-batches it did
 * not finish.  The calling thread is left with the library's device
 * current. */

/* Pin a host range for the library's DMA once (e.g. a server's page pool),
 * so calls on it DMA directly instead of staging.  The range must stay
 * mapped until nkfs_host_unregister; a call in flight holds a reference, so
 * an unregister never unpins under it.  -EEXIST when the runtime already
 * knows the range as pinned (nothing to do), -EBUSY when it partly overlaps
 * a registered range. */
int nkfs_host_register(void *p, size_t bytes);
int nkfs_host_unregister(void *p);
/* Host-path state, for tests and leak checks: out[0] registered ranges,
 * out[1] registry references held by calls in flight, out[2] host lane
 * threads running, out[3] host copy threads running, out[4] per-call
 * contexts (stream + scratch) handed out and not yet returned.  Fills
 * min(n, 5) values; returns 5. */
int nkfs_host_state(uint64_t *out, int n);

/* Host-memory form of nkfs_nk8_encode: blocks, ids, parts and digests in
 * host memory. */
int nkfs_nk8_encode_host(const uint8_t *h_blocks, uint64_t block_pitch,
			 uint32_t block_size, uint32_t nstripes, int n, int k,
			 const uint8_t *h_ids, uint8_t *h_parts,
			 uint64_t part_pitch, uint64_t *h_digests,
			 uint64_t chunk_bytes);

/* Host-memory form of nkfs_nk8_encode_ragged (the C5 mixed batch):
 * stripe s is h_block_size[s] bytes at h_blocks + h_block_off[s], part i
 * goes to h_parts + h_part_off[s] + i*nkfs_part_pitch(h_block_size[s], k)
 * (h_part_off[s] a multiple of 16), digests to h_digests[s*n + i].  Blocks
 * and part ranges must be in increasing order without overlap (gaps are
 * allowed and left untouched); -EINVAL otherwise. */
int nkfs_nk8_encode_ragged_host(const uint8_t *h_blocks,
				const uint64_t *h_block_off,
				const uint32_t *h_block_size,
				uint32_t max_block_size, uint32_t nstripes,
				int n, int k, const uint8_t *h_ids,
				uint8_t *h_parts, const uint64_t *h_part_off,
				uint64_t *h_digests, uint64_t chunk_bytes);

/* PUT from page lists (core/upages.c:91-122: struct nkfs_pages, an array
 * of page pointers): block s is the first h_block_size[s] bytes of pages
 * h_pages[h_first_page[s]], h_pages[h_first_page[s] + 1], ... (page_size
 * bytes each).  Parts and digests as nkfs_nk8_encode_ragged_host. */
int nkfs_nk8_encode_pages(const uint8_t *const *h_pages, uint32_t page_size,
			  const uint64_t *h_first_page, const uint32_t *h_block_size,
			  uint32_t max_block_size, uint32_t nstripes, int n, int k,
			  const uint8_t *h_ids, uint8_t *h_parts,
			  const uint64_t *h_part_off, uint64_t *h_digests,
			  uint64_t chunk_bytes);

/* GET: nkfs_nk8_decode from host memory.  Stripe s's n_slots part slots
 * are at h_parts + (s*n_slots + j)*part_pitch; every slot travels over
 * PCIe, so pass the parts you hold (e.g. the k survivors, n_slots = k).
 * Selection, status (h_status may be NULL) as nkfs_nk8_decode; with
 * h_expect != NULL the part check of nkfs_nk8_decode_verify is fused in
 * (status -EIO, h_badmask may be NULL). */
int nkfs_nk8_decode_host(const uint8_t *h_parts, uint64_t part_pitch, int n_slots,
			 const uint8_t *h_ids, const uint8_t *h_avail, int navail, int k,
			 uint32_t block_size, uint8_t *h_blocks, uint64_t block_pitch,
			 uint32_t nstripes, int32_t *h_status, const uint64_t *h_expect,
			 uint64_t *h_badmask, uint64_t chunk_bytes);

/* GET of a ragged batch: layout of nkfs_nk8_encode_ragged_host with
 * n_slots slots per stripe at h_parts + h_part_off[s] + j*pitch(B_s). */
int nkfs_nk8_decode_ragged_host(const uint8_t *h_parts, const uint64_t *h_part_off,
				int n_slots, const uint8_t *h_ids, const uint8_t *h_avail,
				int navail, int k, uint8_t *h_blocks,
				const uint64_t *h_block_off, const uint32_t *h_block_size,
				uint32_t max_block_size, uint32_t nstripes, int32_t *h_status,
				const uint64_t *h_expect, uint64_t *h_badmask,
				uint64_t chunk_bytes);

/* GET into page lists (the read side of core/net.c:228-265): parts as
 * nkfs_nk8_decode_ragged_host, block s written to its pages as
 * nkfs_nk8_encode_pages reads them. */
int nkfs_nk8_decode_pages(const uint8_t *h_parts, const uint64_t *h_part_off, int n_slots,
			  const uint8_t *h_ids, const uint8_t *h_avail, int navail, int k,
			  uint8_t *const *h_pages, uint32_t page_size,
			  const uint64_t *h_first_page, const uint32_t *h_block_size,
			  uint32_t max_block_size, uint32_t nstripes, int32_t *h_status,
			  const uint64_t *h_expect, uint64_t *h_badmask, uint64_t chunk_bytes);

/* Fill a uniform batch with the seeded counter-based splitmix64 stripes of
 * nkfs_amd/synth.py (bench / test input synthesis on the device). */
int nkfs_synth_blocks(uint8_t *d_blocks, uint64_t block_pitch,
		      uint32_t block_size, uint32_t nstripes, uint64_t seed,
		      uint64_t first_stripe, void *stream);

/* The same stripes for a ragged layout in one launch: stripe s (stripe
 * index first_stripe + s) is d_block_size[s] bytes at d_blocks +
 * d_block_off[s]. */
int nkfs_synth_ragged(uint8_t *d_blocks, const uint64_t *d_block_off,
		      const uint32_t *d_block_size, uint32_t nstripes, uint64_t seed,
		      uint64_t first_stripe, void *stream);

/* Device memory helpers for callers without their own allocator. */
void *nkfs_dev_alloc(size_t bytes);
void nkfs_dev_free(void *d_ptr);
int nkfs_memcpy_h2d(void *d_dst, const void *src, size_t bytes);
int nkfs_memcpy_d2h(void *dst, const void *d_src, size_t bytes);
int nkfs_stream_sync(void *stream);

#ifdef __cplusplus
}
#endif
#endif
