/*
 * runtime.c -- device context of libnkfs_crt.so and the batched C-ABI of
 * include/nkfs_gpu.h.  Host C over the HIP runtime; every computation is a
 * kernel launched through nkfs_internal.h.
 *
 * State: the library's device (chosen at init: the compatibility entry
 * points run there), and per device a copy of the GF(2^8) log/antilog
 * tables plus a pool of per-call contexts (stream + growable device/pinned
 * scratch), so that every entry point is reentrant and thread-safe after
 * init like the reference's (SURVEY.md §8(b) "Threading").  Batched device
 * calls run on the device of the caller's stream; the host-memory entry
 * points spread a batch over the device lanes of nkfs_gpu_set_devices.
 */
#include <errno.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "../../include/nkfs_gpu.h"
#include "nkfs_internal.h"
#include "runtime.h"

static pthread_mutex_t g_lock = PTHREAD_MUTEX_INITIALIZER;
static int g_ready;
static int g_device = -1; /* the library's device: compatibility entry points run here */
static int g_cus = 256;

/* Per-device state: GF tables and an idle pool of per-call contexts.  A
 * device is set up on first use (nkfs_gpu_init for the library's device,
 * nkfs_gpu_set_devices or a batched call on another device's stream). */
struct nkfs_dev {
	int ready;
	void *gf;
	struct nkfs_ctx *pool;
};
static struct nkfs_dev g_dev[NKFS_MAX_DEVICES];

/* Devices the host-memory entry points spread a batch over (one lane per
 * entry, repeats allowed); empty = the library's device. */
static int g_lanes[NKFS_MAX_DEVICES];
static int g_nlanes;

/* Measured defaults; nkfs_tune_set replaces them.  Read
 * and written only under g_tune_lock: every launch takes one consistent
 * copy (nkfs_tune_now), so a concurrent nkfs_tune_set never tears a read. */
static pthread_mutex_t g_tune_lock = PTHREAD_MUTEX_INITIALIZER;
static struct nkfs_tune g_tune = {
	.enc_kernel = NKFS_ENC_AUTO,
	.dec_kernel = NKFS_DEC_AUTO,
	.enc_waves_per_cu = 8,
	.dec_waves_per_cu = 12,
	.dec_units = 2,
	.enc_nib = -1,
	.enc_units = 0,
	.size_order = 1,
	.enc_prefetch = 1,
	.enc_fused_waves_per_cu = 0,
	.dec_wave_waves_per_cu = 0,
	.dec_run_units = 4,
	.enc_ws_prefetch = 2, /* W1 encode 3,952 -> 4,043 GB/s, N16K10 +0.9 %, C3 / C4 even (profiles/r04/ab_wide_nib.txt) */
	.dec_pair_stage = 1,
	.host_depth = 6,  /* C3 1 GiB PUT / GET: 17.2 / 27.6 GiB/s at 3 x 1, 21.5 / 34.1 at 6 x 2 */
	.host_lanes = 2,  /* (profiles/r04/pcie.txt) */
	.enc_ws_waves = 4,
	.enc_few_max = 63,
	.enc_ws_hash_waves = 0, /* auto: 2 from 1,024 stripes (profiles/r04/seam_ws2.txt) */
	.enc_persist = 1, /* ragged n > 4: C5 encode 4,839 -> 5,051 GB/s (profiles/r05/ab_wsp.txt) */
	.dec_bign = -2, /* auto: byte tables for k % 4 == 0 (not 16), all-groups form for the other 16 < k <= 64
	                 * (profiles/r05/ab_bign.txt, profiles/r06/ab_bigr_*.txt, ab_rule_k*.txt) */
	.enc_bign = -1,
	.enc_big_fused = -1, /* auto: the XXH64 pass (round 6: W3 +10 % over the fused chain with diagonal tables; profiles/r06/ab_w3_enc.txt) */
	.dec_pair_pipe = 0,
	.dec_pair_waves = 1, /* C2: 1 wave per workgroup 5,214 / 4 waves 5,116 GB/s (profiles/r04/ab_c2_pair4.txt) */
};

void nkfs_tune_get(struct nkfs_tune *t)
{
	if (!t)
		return;
	pthread_mutex_lock(&g_tune_lock);
	*t = g_tune;
	pthread_mutex_unlock(&g_tune_lock);
}

int nkfs_tune_set(const struct nkfs_tune *t)
{
	if (!t || t->enc_kernel < NKFS_ENC_AUTO || t->enc_kernel > NKFS_ENC_WSP || t->dec_kernel < NKFS_DEC_AUTO ||
	    t->dec_kernel > NKFS_DEC_PAIR || t->enc_waves_per_cu < 1 || t->enc_waves_per_cu > 32 ||
	    t->dec_waves_per_cu < 1 || t->dec_waves_per_cu > 32 ||
	    (t->dec_units != 1 && t->dec_units != 2 && t->dec_units != 4) || t->enc_nib < -1 || t->enc_nib > 1 ||
	    t->enc_units < 0 || t->enc_units > 2 ||
	    (t->size_order != 0 && t->size_order != 1) || t->enc_prefetch < 1 || t->enc_prefetch > 2 ||
	    (t->enc_fused_waves_per_cu && (t->enc_fused_waves_per_cu < 3 || t->enc_fused_waves_per_cu > 32)) ||
	    (t->dec_wave_waves_per_cu && (t->dec_wave_waves_per_cu < 3 || t->dec_wave_waves_per_cu > 32)) ||
	    (t->dec_run_units != 1 && t->dec_run_units != 2 && t->dec_run_units != 4 && t->dec_run_units != 8 &&
	     t->dec_run_units != 16) ||
	    t->enc_ws_prefetch < 1 || t->enc_ws_prefetch > 2 || (t->enc_big_fused < -1 || t->enc_big_fused > 1) ||
	    (t->dec_pair_stage != 0 && t->dec_pair_stage != 1) || t->host_depth < 2 || t->host_depth > 8 ||
	    t->host_lanes < 1 || t->host_lanes > 4 || t->enc_ragged_split < 0 ||
	    (t->enc_ws_waves != 4 && t->enc_ws_waves != 6) || (t->dec_pair_waves != 1 && t->dec_pair_waves != 4) ||
	    t->enc_few_max < 0 || t->enc_few_max > 63 || t->enc_ws_hash_waves < 0 || t->enc_ws_hash_waves > 2 ||
	    t->enc_persist < 0 || t->enc_persist > 2 ||
	    t->dec_bign < -2 || t->dec_bign > 5 || t->enc_bign < -1 || t->enc_bign > 3 ||
	    t->dec_pair_pipe < 0 || t->dec_pair_pipe > 32)
		return -EINVAL;
	pthread_mutex_lock(&g_tune_lock);
	g_tune = *t;
	pthread_mutex_unlock(&g_tune_lock);
	return 0;
}

int nkfs_host_depth(void)
{
	struct nkfs_tune t;
	nkfs_tune_get(&t);
	return t.host_depth;
}

int nkfs_host_lanes(void)
{
	struct nkfs_tune t;
	nkfs_tune_get(&t);
	return t.host_lanes;
}

int nkfs_hip_fail(const char *what, int err)
{
	fprintf(stderr, "nkfs: %s failed: %s\n", what, hipGetErrorString((hipError_t)err));
	return -EIO;
}

#define HIPCHK(call)                                                 \
	do {                                                         \
		hipError_t e_ = (call);                              \
		if (e_ != hipSuccess)                                \
			return nkfs_hip_fail(#call, (int)e_);        \
	} while (0)

/* make `dev` the calling thread's current device (no call when it already is) */
int nkfs_use_device(int dev)
{
	int cur = -1;
	if (hipGetDevice(&cur) == hipSuccess && cur == dev)
		return 0;
	return hipSetDevice(dev) == hipSuccess ? 0 : -EIO;
}

/* GF tables on `dev`, under g_lock.  Leaves `dev` current. */
static int dev_setup_locked(int dev)
{
	struct nkfs_dev *d = &g_dev[dev];
	if (__atomic_load_n(&d->ready, __ATOMIC_ACQUIRE))
		return nkfs_use_device(dev);
	hipError_t e = hipSetDevice(dev);
	if (e == hipSuccess)
		e = hipMalloc(&d->gf, nkfs_gf_tables_bytes());
	if (e != hipSuccess)
		return nkfs_hip_fail("device setup", (int)e);
	int rc = nkfs_launch_gf_init(d->gf, NULL);
	if (!rc && (e = hipDeviceSynchronize()) != hipSuccess)
		rc = nkfs_hip_fail("gf table build", (int)e);
	if (rc) {
		hipFree(d->gf);
		d->gf = NULL;
		return rc;
	}
	/* publish: gf is written before ready reads 1 (nkfs_gf_on reads ready
	 * outside the lock) */
	__atomic_store_n(&d->ready, 1, __ATOMIC_RELEASE);
	return 0;
}

static int device_count(void)
{
	int count = 0;
	if (hipGetDeviceCount(&count) != hipSuccess)
		return 0;
	return count < NKFS_MAX_DEVICES ? count : NKFS_MAX_DEVICES;
}

int nkfs_gpu_init(int device)
{
	int rc = 0;
	pthread_mutex_lock(&g_lock);
	if (g_ready)
		goto out;
	int count = device_count();
	if (count <= 0) {
		fprintf(stderr, "nkfs: no HIP device visible; the MI355X path has no CPU fallback\n");
		rc = -ENODEV;
		goto out;
	}
	if (device < 0) {
		const char *env = getenv("NKFS_DEVICE");
		if (env && *env)
			device = atoi(env);
		else if (hipGetDevice(&device) != hipSuccess)
			device = 0;
	}
	if (device < 0 || device >= count) {
		rc = -ENODEV;
		goto out;
	}
	if ((rc = dev_setup_locked(device)))
		goto out;
	int cus = 0;
	if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
		g_cus = cus;
	g_device = device;
	__atomic_store_n(&g_ready, 1, __ATOMIC_RELEASE); /* after g_device, g_cus */
out:
	pthread_mutex_unlock(&g_lock);
	return rc;
}

static int ready_now(void) { return __atomic_load_n(&g_ready, __ATOMIC_ACQUIRE); }

int nkfs_gpu_ready(void) { return ready_now(); }

int nkfs_gpu_device(void) { return ready_now() ? g_device : -1; }

int nkfs_gpu_count(void) { return device_count(); }

int nkfs_cu_count(void) { return g_cus; }

/* GF tables of `dev`, set up on first use; NULL when it cannot be. */
const void *nkfs_gf_on(int dev)
{
	if (dev < 0 || dev >= NKFS_MAX_DEVICES)
		return NULL;
	if (__atomic_load_n(&g_dev[dev].ready, __ATOMIC_ACQUIRE))
		return g_dev[dev].gf;
	pthread_mutex_lock(&g_lock);
	int cur = -1;
	(void)hipGetDevice(&cur);
	int rc = dev < device_count() ? dev_setup_locked(dev) : -ENODEV;
	if (cur >= 0)
		nkfs_use_device(cur);
	pthread_mutex_unlock(&g_lock);
	return rc ? NULL : g_dev[dev].gf;
}

/* GF tables of the device a launch on `stream` runs on (NULL stream: the
 * calling thread's current device). */
const void *nkfs_gf_for(void *stream)
{
	int dev = -1;
	if (stream) {
		if (hipStreamGetDevice((hipStream_t)stream, &dev) != hipSuccess)
			return NULL;
	} else if (hipGetDevice(&dev) != hipSuccess) {
		return NULL;
	}
	return nkfs_gf_on(dev);
}

const void *nkfs_gf(void) { return ready_now() ? g_dev[g_device].gf : NULL; }

int nkfs_gpu_set_devices(const int *devices, int count)
{
	if (count < 0 || count > NKFS_MAX_DEVICES || (count && !devices))
		return -EINVAL;
	if (!ready_now())
		return -EAGAIN;
	const int ndev = device_count();
	for (int i = 0; i < count; i++)
		if (devices[i] < 0 || devices[i] >= ndev)
			return -ENODEV;
	int rc = 0;
	pthread_mutex_lock(&g_lock);
	int cur = -1;
	(void)hipGetDevice(&cur);
	for (int i = 0; i < count && !rc; i++)
		rc = dev_setup_locked(devices[i]);
	if (!rc) {
		for (int i = 0; i < count; i++)
			g_lanes[i] = devices[i];
		g_nlanes = count;
	}
	if (cur >= 0)
		nkfs_use_device(cur);
	pthread_mutex_unlock(&g_lock);
	return rc;
}

int nkfs_gpu_get_devices(int *devices, int max)
{
	pthread_mutex_lock(&g_lock);
	int n = g_nlanes ? g_nlanes : (ready_now() ? 1 : 0);
	for (int i = 0; i < n && i < max && devices; i++)
		devices[i] = g_nlanes ? g_lanes[i] : g_device;
	pthread_mutex_unlock(&g_lock);
	return n;
}

static void ctx_destroy(struct nkfs_ctx *c)
{
	hipStreamSynchronize(c->stream);
	for (int i = 0; i < c->nev; i++)
		hipEventDestroy(c->ev[i]);
	hipStreamDestroy(c->stream);
	hipFree(c->dbuf);
	hipHostFree(c->hbuf);
	if (c->done)
		hipHostFree((void *)c->done);
	free(c);
}

static void pools_drain(struct nkfs_ctx **taken)
{
	for (int d = 0; d < NKFS_MAX_DEVICES; d++) {
		struct nkfs_ctx *pool = taken[d];
		if (!pool)
			continue;
		hipSetDevice(d);
		while (pool) {
			struct nkfs_ctx *c = pool;
			pool = c->next;
			ctx_destroy(c);
		}
	}
}

void nkfs_gpu_release(void)
{
	struct nkfs_ctx *taken[NKFS_MAX_DEVICES] = {0};
	pthread_mutex_lock(&g_lock);
	for (int d = 0; d < NKFS_MAX_DEVICES; d++) {
		taken[d] = g_dev[d].pool;
		g_dev[d].pool = NULL;
	}
	pools_drain(taken);
	for (int d = 0; d < NKFS_MAX_DEVICES; d++)
		if (g_dev[d].ready) {
			hipSetDevice(d);
			hipFree(g_dev[d].gf);
			g_dev[d].gf = NULL;
			__atomic_store_n(&g_dev[d].ready, 0, __ATOMIC_RELEASE);
		}
	__atomic_store_n(&g_ready, 0, __ATOMIC_RELEASE);
	g_nlanes = 0;
	pthread_mutex_unlock(&g_lock);
}

void nkfs_ctx_trim(void)
{
	struct nkfs_ctx *taken[NKFS_MAX_DEVICES] = {0};
	pthread_mutex_lock(&g_lock);
	for (int d = 0; d < NKFS_MAX_DEVICES; d++) {
		taken[d] = g_dev[d].pool;
		g_dev[d].pool = NULL;
	}
	pthread_mutex_unlock(&g_lock);
	pools_drain(taken);
	if (ready_now())
		nkfs_use_device(g_device);
}

/* A per-call context (stream + scratch) on `dev`, from its idle pool or new;
 * leaves `dev` current for the calling thread. */
static uint64_t g_ctx_out; /* contexts handed out (atomics; nkfs_host_state) */

uint64_t nkfs_ctx_outstanding(void)
{
	return __atomic_load_n(&g_ctx_out, __ATOMIC_RELAXED);
}

struct nkfs_ctx *nkfs_ctx_get_on(int dev)
{
	struct nkfs_ctx *c = NULL;
	if (!ready_now() || dev < 0 || dev >= NKFS_MAX_DEVICES || !nkfs_gf_on(dev))
		return NULL;
	pthread_mutex_lock(&g_lock);
	if (g_dev[dev].pool) {
		c = g_dev[dev].pool;
		g_dev[dev].pool = c->next;
	}
	pthread_mutex_unlock(&g_lock);
	if (nkfs_use_device(dev))
		goto fail;
	if (!c) {
		c = calloc(1, sizeof(*c));
		if (!c)
			return NULL;
		c->dev = dev;
		if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
			goto fail;
	}
	__atomic_add_fetch(&g_ctx_out, 1, __ATOMIC_RELAXED);
	return c;
fail:
	if (c) {
		__atomic_add_fetch(&g_ctx_out, 1, __ATOMIC_RELAXED); /* nkfs_ctx_put takes it back */
		nkfs_ctx_put(c);
	}
	return NULL;
}

struct nkfs_ctx *nkfs_ctx_get(void)
{
	return ready_now() ? nkfs_ctx_get_on(g_device) : NULL;
}

#define POOL_KEEP 32 /* >= host_lanes x host_depth at their maxima */

void nkfs_ctx_put(struct nkfs_ctx *c)
{
	if (!c)
		return;
	__atomic_sub_fetch(&g_ctx_out, 1, __ATOMIC_RELAXED);
	if (!c->stream) {
		free(c);
		return;
	}
	/* the idle pool keeps at most POOL_KEEP contexts per device: a burst
	 * (many pending checksum states, many concurrent host calls) does not
	 * hold its streams and pinned / device scratch for the process's life */
	int n = 0;
	pthread_mutex_lock(&g_lock);
	for (struct nkfs_ctx *e = g_dev[c->dev].pool; e; e = e->next)
		n++;
	if (n < POOL_KEEP) {
		c->next = g_dev[c->dev].pool;
		g_dev[c->dev].pool = c;
		c = NULL;
	}
	pthread_mutex_unlock(&g_lock);
	if (c) {
		int cur = -1;
		(void)hipGetDevice(&cur);
		nkfs_use_device(c->dev);
		ctx_destroy(c);
		if (cur >= 0)
			nkfs_use_device(cur);
	}
}

int nkfs_ctx_dev(struct nkfs_ctx *c, size_t bytes, void **out)
{
	if (bytes > c->dcap) {
		hipStreamSynchronize(c->stream);
		hipFree(c->dbuf);
		c->dbuf = NULL;
		c->dcap = 0;
		size_t cap = bytes < (1u << 20) ? (1u << 20) : bytes;
		HIPCHK(hipMalloc(&c->dbuf, cap));
		c->dcap = cap;
	}
	*out = c->dbuf;
	return 0;
}

int nkfs_ctx_events(struct nkfs_ctx *c)
{
	while (c->nev < 2) {
		HIPCHK(hipEventCreateWithFlags(&c->ev[c->nev], hipEventDisableTiming));
		c->nev++;
	}
	return 0;
}

/* Wait for the context's stream to drain without hipStreamSynchronize: the
 * stream writes the next sequence number to a pinned word once all earlier
 * work is done (hipStreamWriteValue64 orders after it, the kernels' host
 * writes released at system scope), and the host spins on that word.  The
 * stream's status is polled now and then, so a failed launch cannot spin
 * forever.  The one-block drop-in calls wait here: the extra stream packet
 * costs ~4 us on a 4 KiB call, where the stream sync still spins, but the
 * sync's later wake-up costs 2-28 us from 64 KiB blocks on
 * (profiles/r04/percall_spin_vs_sync.txt), so callers spin from 32 KiB. */
/* pause iterations a completion wait spins before it blocks (~1-2 ms) */
#define NKFS_SPIN_MAX (16ull << 16)

int nkfs_ctx_wait(struct nkfs_ctx *c, int spin)
{
#ifdef NKFS_WAIT_SYNC /* A/B builds: the plain stream sync */
	spin = 0;
#endif
	if (!spin) {
		HIPCHK(hipStreamSynchronize(c->stream));
		return 0;
	}
	if (!c->done) {
		void *h = NULL, *d = NULL;
		HIPCHK(hipHostMalloc(&h, 64, hipHostMallocDefault));
		if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
			hipHostFree(h);
			return -EIO;
		}
		memset(h, 0, 64);
		c->done = h;
		c->ddone = d;
	}
	const uint64_t want = ++c->seq;
	if (hipStreamWriteValue64(c->stream, c->ddone, want, 0) != hipSuccess) {
		(void)hipGetLastError();
		HIPCHK(hipStreamSynchronize(c->stream));
		return 0;
	}
	/* spin on the completion word for a bounded time (a small call's late
	 * stream-sync wake-up costs more than the call), then block in the
	 * stream sync instead of burning a core for a long one */
	for (uint64_t it = 0; __atomic_load_n(c->done, __ATOMIC_ACQUIRE) != want; it++) {
		if ((it & 0xFFFF) == 0xFFFF) {
			hipError_t q = hipStreamQuery(c->stream);
			if (q != hipSuccess && q != hipErrorNotReady)
				return nkfs_hip_fail("hipStreamQuery", (int)q);
			if (q == hipSuccess && __atomic_load_n(c->done, __ATOMIC_ACQUIRE) != want)
				return -EIO; /* the stream drained without the word */
			if (it >= NKFS_SPIN_MAX) {
				HIPCHK(hipStreamSynchronize(c->stream));
				if (__atomic_load_n(c->done, __ATOMIC_ACQUIRE) != want)
					return -EIO;
				break;
			}
		}
		__builtin_ia32_pause();
	}
	return 0;
}

int nkfs_ctx_host(struct nkfs_ctx *c, size_t bytes, void **out)
{
	if (bytes > c->hcap) {
		hipStreamSynchronize(c->stream);
		hipHostFree(c->hbuf);
		c->hbuf = NULL;
		c->hcap = 0;
		size_t cap = bytes < (1u << 16) ? (1u << 16) : bytes;
		HIPCHK(hipHostMalloc(&c->hbuf, cap, hipHostMallocDefault));
		c->hcap = cap;
	}
	*out = c->hbuf;
	return 0;
}

/* ------------------------------------------------------------ batch API */

uint32_t nkfs_part_size(uint32_t block_size, int k)
{
	if (k <= 0)
		return 0;
	return block_size / (uint32_t)k + ((block_size % (uint32_t)k) ? 1u : 0u);
}

uint64_t nkfs_part_pitch(uint32_t block_size, int k)
{
	return ((uint64_t)nkfs_part_size(block_size, k) + NKFS_PART_ALIGN - 1) & ~(uint64_t)(NKFS_PART_ALIGN - 1);
}

/* crt/nk8.c:356-360: 2 <= k <= n <= 255, k <= 254, block_size > 0 */
int nkfs_bad_params(uint32_t block_size, int n, int k)
{
	return n < 2 || k < 2 || block_size == 0 || n < k || n > 255 || k > 254;
}

int nkfs_nk8_encode(const uint8_t *d_blocks, uint64_t block_pitch, uint32_t block_size, uint32_t nstripes,
		    int n, int k, const uint8_t *d_ids, uint8_t *d_parts, uint64_t part_pitch, uint64_t *d_digests,
		    void *stream)
{
	if (nkfs_bad_params(block_size, n, k))
		return -EINVAL;
	if (!ready_now())
		return -EAGAIN;
	if (!nstripes)
		return 0;
	if (!d_blocks || !d_ids || !d_parts || part_pitch < nkfs_part_size(block_size, k) || (part_pitch & 15) ||
	    (nstripes > 1 && block_pitch < block_size))
		return -EINVAL;
	const void *gf = nkfs_gf_for(stream);
	if (!gf)
		return -ENODEV;
	struct nkfs_geom g = { d_blocks, block_pitch, block_size, NULL, NULL, d_parts, part_pitch, NULL,
			       nstripes, n, k, NULL, 0, 0, NULL, 0, 0, 0, NULL };
	return nkfs_launch_encode(&g, d_ids, d_digests, gf, stream);
}

int nkfs_nk8_encode_ragged(const uint8_t *d_blocks, const uint64_t *d_block_off, const uint32_t *d_block_size,
			   uint32_t max_block_size, uint32_t nstripes, int n, int k, const uint8_t *d_ids,
			   uint8_t *d_parts, const uint64_t *d_part_off, uint64_t *d_digests, void *stream)
{
	if (nkfs_bad_params(max_block_size, n, k))
		return -EINVAL;
	if (!ready_now())
		return -EAGAIN;
	if (!nstripes)
		return 0;
	if (!d_blocks || !d_block_off || !d_block_size || !d_ids || !d_parts || !d_part_off)
		return -EINVAL;
	const void *gf = nkfs_gf_for(stream);
	if (!gf)
		return -ENODEV;
	struct nkfs_geom g = { d_blocks, 0, max_block_size, d_block_off, d_block_size, d_parts, 0, d_part_off,
			       nstripes, n, k, NULL, 0, 0, NULL, 0, 0, 0, NULL };
	return nkfs_launch_encode(&g, d_ids, d_digests, gf, stream);
}

uint64_t nkfs_decode_workspace(uint32_t nstripes, int k)
{
	return nkfs_decode_work_bytes(nstripes, k);
}

static int decode_common(const uint8_t *d_parts, uint64_t part_pitch, int n_slots, const uint8_t *d_ids,
			 const uint8_t *d_avail, int navail, int k, uint32_t block_size, uint8_t *d_blocks,
			 uint64_t block_pitch, uint32_t nstripes, void *d_work, int32_t *d_status,
			 const uint64_t *d_expect, uint64_t *d_badmask, void *stream)
{
	if (nkfs_bad_params(block_size, navail, k) || n_slots < 1 || n_slots > 255)
		return -EINVAL;
	if (!ready_now())
		return -EAGAIN;
	if (!nstripes)
		return 0;
	if (!d_parts || !d_ids || !d_avail || !d_blocks || !d_work || part_pitch < nkfs_part_size(block_size, k) ||
	    (nstripes > 1 && block_pitch < block_size))
		return -EINVAL;
	const void *gf = nkfs_gf_for(stream);
	if (!gf)
		return -ENODEV;
	struct nkfs_geom g = { d_blocks, block_pitch, block_size, NULL, NULL, (uint8_t *)d_parts, part_pitch, NULL,
			       nstripes, n_slots, k, NULL, 0, 0, NULL, 0, 0, 0, NULL };
	return nkfs_launch_decode(&g, n_slots, d_ids, d_avail, navail, d_work, d_status, gf, stream, d_expect,
				  d_badmask);
}

int nkfs_nk8_decode(const uint8_t *d_parts, uint64_t part_pitch, int n_slots, const uint8_t *d_ids,
		    const uint8_t *d_avail, int navail, int k, uint32_t block_size, uint8_t *d_blocks,
		    uint64_t block_pitch, uint32_t nstripes, void *d_work, int32_t *d_status, void *stream)
{
	return decode_common(d_parts, part_pitch, n_slots, d_ids, d_avail, navail, k, block_size, d_blocks,
			     block_pitch, nstripes, d_work, d_status, NULL, NULL, stream);
}

static int decode_ragged_common(const uint8_t *d_parts, const uint64_t *d_part_off, int n_slots,
				const uint8_t *d_ids, const uint8_t *d_avail, int navail, int k, uint8_t *d_blocks,
				const uint64_t *d_block_off, const uint32_t *d_block_size, uint32_t max_block_size,
				uint32_t nstripes, void *d_work, int32_t *d_status, const uint64_t *d_expect,
				uint64_t *d_badmask, void *stream)
{
	if (nkfs_bad_params(max_block_size, navail, k) || n_slots < 1 || n_slots > 255)
		return -EINVAL;
	if (!ready_now())
		return -EAGAIN;
	if (!nstripes)
		return 0;
	if (!d_parts || !d_part_off || !d_ids || !d_avail || !d_blocks || !d_block_off || !d_block_size || !d_work)
		return -EINVAL;
	const void *gf = nkfs_gf_for(stream);
	if (!gf)
		return -ENODEV;
	struct nkfs_geom g = { d_blocks, 0, max_block_size, d_block_off, d_block_size, (uint8_t *)d_parts, 0,
			       d_part_off, nstripes, n_slots, k, NULL, 0, 0, NULL, 0, 0, 0, NULL };
	return nkfs_launch_decode(&g, n_slots, d_ids, d_avail, navail, d_work, d_status, gf, stream, d_expect,
				  d_badmask);
}

int nkfs_nk8_decode_ragged(const uint8_t *d_parts, const uint64_t *d_part_off, int n_slots, const uint8_t *d_ids,
			   const uint8_t *d_avail, int navail, int k, uint8_t *d_blocks, const uint64_t *d_block_off,
			   const uint32_t *d_block_size, uint32_t max_block_size, uint32_t nstripes, void *d_work,
			   int32_t *d_status, void *stream)
{
	return decode_ragged_common(d_parts, d_part_off, n_slots, d_ids, d_avail, navail, k, d_blocks, d_block_off,
				    d_block_size, max_block_size, nstripes, d_work, d_status, NULL, NULL, stream);
}

int nkfs_nk8_decode_ragged_verify(const uint8_t *d_parts, const uint64_t *d_part_off, int n_slots,
				  const uint8_t *d_ids, const uint8_t *d_avail, int navail, int k, uint8_t *d_blocks,
				  const uint64_t *d_block_off, const uint32_t *d_block_size, uint32_t max_block_size,
				  uint32_t nstripes, void *d_work, int32_t *d_status, const uint64_t *d_expect,
				  uint64_t *d_badmask, void *stream)
{
	if (!d_expect)
		return -EINVAL;
	return decode_ragged_common(d_parts, d_part_off, n_slots, d_ids, d_avail, navail, k, d_blocks, d_block_off,
				    d_block_size, max_block_size, nstripes, d_work, d_status, d_expect, d_badmask,
				    stream);
}

int nkfs_nk8_decode_verify(const uint8_t *d_parts, uint64_t part_pitch, int n_slots, const uint8_t *d_ids,
			   const uint8_t *d_avail, int navail, int k, uint32_t block_size, uint8_t *d_blocks,
			   uint64_t block_pitch, uint32_t nstripes, void *d_work, int32_t *d_status,
			   const uint64_t *d_expect, uint64_t *d_badmask, void *stream)
{
	if (!d_expect)
		return -EINVAL;
	return decode_common(d_parts, part_pitch, n_slots, d_ids, d_avail, navail, k, block_size, d_blocks,
			     block_pitch, nstripes, d_work, d_status, d_expect, d_badmask, stream);
}

int nkfs_xxh64_batch(const uint8_t *d_base, const uint64_t *d_off, const uint64_t *d_len, uint32_t count,
		     uint64_t seed, uint64_t *d_out, void *stream)
{
	if (!ready_now())
		return -EAGAIN;
	if (count && (!d_base || !d_off || !d_len || !d_out))
		return -EINVAL;
	return nkfs_launch_xxh64_batch(d_base, d_off, d_len, count, seed, d_out, stream);
}

int nkfs_clu_sum_batch(const uint8_t *d_clusters, uint64_t cluster_pitch, uint32_t cluster_size, uint32_t count,
		       uint64_t *d_sums, const uint64_t *d_expect, int32_t *d_status, void *stream)
{
	if (!ready_now())
		return -EAGAIN;
	if (!count)
		return 0;
	if (!d_clusters || !d_sums || (d_expect && !d_status) || ((uintptr_t)d_clusters & 7) ||
	    (count > 1 && (cluster_pitch < cluster_size || (cluster_pitch & 7))))
		return -EINVAL;
	return nkfs_fast_xxh64_strided(d_clusters, cluster_pitch, cluster_size, count, d_sums, d_expect, d_status,
				       stream);
}

int nkfs_pages_dsum_batch(const uint8_t *const *d_pages, const uint64_t *d_first_page, const uint64_t *d_len,
			  uint32_t count, uint32_t page_size, uint64_t *d_dsums, void *stream)
{
	uint32_t shift = 0;

	if (!ready_now())
		return -EAGAIN;
	if (!count)
		return 0;
	if (!d_pages || !d_first_page || !d_len || !d_dsums)
		return -EINVAL;
	/* a 512-byte hashing chunk must never straddle two pages */
	if (page_size < 512 || (page_size & (page_size - 1)))
		return -EINVAL;
	while ((1u << shift) < page_size)
		shift++;
	return nkfs_fast_xxh64_pages(d_pages, d_first_page, d_len, count, shift, d_dsums, stream);
}

int nkfs_synth_blocks(uint8_t *d_blocks, uint64_t block_pitch, uint32_t block_size, uint32_t nstripes,
		      uint64_t seed, uint64_t first_stripe, void *stream)
{
	if (!ready_now())
		return -EAGAIN;
	if (nstripes && (!d_blocks || (nstripes > 1 && block_pitch < block_size)))
		return -EINVAL;
	return nkfs_launch_synth(d_blocks, block_pitch, block_size, nstripes, seed, first_stripe, stream);
}

int nkfs_synth_ragged(uint8_t *d_blocks, const uint64_t *d_block_off, const uint32_t *d_block_size,
		      uint32_t nstripes, uint64_t seed, uint64_t first_stripe, void *stream)
{
	if (!ready_now())
		return -EAGAIN;
	if (nstripes && (!d_blocks || !d_block_off || !d_block_size))
		return -EINVAL;
	return nkfs_launch_synth_ragged(d_blocks, d_block_off, d_block_size, nstripes, seed, first_stripe, stream);
}

void *nkfs_dev_alloc(size_t bytes)
{
	void *p = NULL;
	if (!ready_now() || nkfs_use_device(g_device) || hipMalloc(&p, bytes ? bytes : 1) != hipSuccess)
		return NULL;
	return p;
}

void nkfs_dev_free(void *p)
{
	if (p)
		hipFree(p);
}

int nkfs_memcpy_h2d(void *dst, const void *src, size_t bytes)
{
	HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
	return 0;
}

int nkfs_memcpy_d2h(void *dst, const void *src, size_t bytes)
{
	HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
	return 0;
}

int nkfs_stream_sync(void *stream)
{
	HIPCHK(hipStreamSynchronize((hipStream_t)stream));
	return 0;
}

/* ------------------------------------------------------------- memory */

void *crt_malloc(size_t size) { return malloc(size); }
void crt_free(void *ptr) { free(ptr); }
