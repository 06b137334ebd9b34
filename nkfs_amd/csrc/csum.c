/*
 * csum.c -- the reference's checksum ABI (crt/include/csum.h:14-17,
 * crt/include/xxhash.h:86-132; XXH32 is not on the path and not exported)
 * with the XXH64 rounds, merge, tail and avalanche computed on the GPU
 * (k_xxh64_chain, xxh64_chain.hip: one wave, the message's four serial
 * chains at round latency, reading the staged bytes from pinned host memory).
 *
 * The state keeps the reference's internal layout (crt/xxhash.c:515-525)
 * inside the caller-owned 88-byte XXH64_state_t, and the host side does what
 * the reference's update does with memory: it buffers an incomplete 32-byte
 * stripe in mem64 (crt/xxhash.c:750-770, 823-833).
 *
 * One GPU round trip per message.  XXH64_update does not wait for the GPU:
 * whole stripes are copied into pinned staging of a per-message context
 * (stream + staging + device accumulators) held in a slot; every full
 * 256 KiB of staging is folded by an asynchronous launch (accumulators stay
 * on the device), so a long stream overlaps the host's copy with the GPU's
 * chains.  XXH64_digest launches the last fold together with merge, tail
 * and avalanche and spins on a completion word the kernel stores to host
 * memory -- no stream synchronisation -- then writes the accumulators back
 * into the state (the reference's state after the same updates) and frees
 * the slot.  XXH64() / csum_* are reset + update + digest: one launch for
 * messages up to 256 KiB.
 *
 * While a message is pending, the state's padding word (offset 84 of the
 * 88 bytes, unused by the reference layout) holds the slot, and v[0] a
 * 64-bit token of it; byte-copying a pending state and continuing both
 * copies is not supported (the copy that digests second traps like
 * CRT_BUG instead of returning a wrong sum).  When all slots are taken an
 * update folds synchronously (one round trip) instead.
 *
 * These per-call entry points keep drop-in callers (client/lib/client.c,
 * crt/net_pkt.c) working; high-volume hashing belongs in
 * nkfs_xxh64_batch / the fused encode (include/nkfs_gpu.h).
 */
#include <errno.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/nkfs_crt.h"
#include "../../include/nkfs_gpu.h"
#include "nkfs_internal.h"
#include "runtime.h"

struct xstate {           /* crt/xxhash.c:515-525, + the pending word in the padding */
	uint64_t total_len;
	uint64_t seed;
	uint64_t v[4];
	uint64_t mem64[4];
	uint32_t memsize;
	uint32_t pend;    /* PEND_MAGIC | slot while a message is on the GPU */
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
	XXH64_state_t *st = crt_malloc(sizeof(XXH64_state_t));
	if (st)
		memset(st, 0, sizeof(*st));
	return st;
}

/* ------------------------------------------------------ message engine */

#define XH_CHUNK (256u << 10) /* staged bytes (whole stripes) per fold launch */
#define XH_RES 64u            /* pinned result words ahead of the staging */

struct xh {
	struct nkfs_ctx *c;
	uint8_t *res;             /* pinned: [digest, flag, v0..v3] */
	uint64_t *dres;           /* its device-visible address */
	uint8_t *stage[2];
	const uint8_t *dstage[2];
	int cur;
	int inflight[2];          /* a fold reads stage[b] until ev[b] */
	uint32_t fill;            /* bytes staged in stage[cur] */
	int folded;               /* accumulators live on the device */
	uint64_t *v_dev;
	uint64_t v0[4];           /* accumulators when the message started */
};

static int xh_begin(struct xh *h, const uint64_t v[4])
{
	memset(h, 0, sizeof(*h));
	if (ensure_gpu())
		return -ENODEV;
	h->c = nkfs_ctx_get();
	if (!h->c)
		return -EIO;
	void *hv, *dv, *dp;
	int err;
	if ((err = nkfs_ctx_host(h->c, XH_RES + 2 * XH_CHUNK, &hv)) || (err = nkfs_ctx_dev(h->c, 64, &dv)) ||
	    (err = nkfs_ctx_events(h->c)))
		goto fail;
	if (hipHostGetDevicePointer(&dp, hv, 0) != hipSuccess) {
		err = -EIO;
		goto fail;
	}
	h->res = hv;
	h->dres = dp;
	h->stage[0] = (uint8_t *)hv + XH_RES;
	h->stage[1] = h->stage[0] + XH_CHUNK;
	h->dstage[0] = (const uint8_t *)dp + XH_RES;
	h->dstage[1] = h->dstage[0] + XH_CHUNK;
	h->v_dev = dv;
	memcpy(h->v0, v, 32);
	return 0;
fail:
	nkfs_ctx_put(h->c);
	h->c = NULL;
	return err;
}

static void xh_end(struct xh *h)
{
	if (h->c) {
		/* folds still reading the staging finish before the context is reused */
		for (int b = 0; b < 2; b++)
			if (h->inflight[b])
				(void)hipEventSynchronize(h->c->ev[b]);
		nkfs_ctx_put(h->c);
	}
	h->c = NULL;
}

static void xh_args(const struct xh *h, struct nkfs_xxh_args *a, uint32_t flags)
{
	memset(a, 0, sizeof(*a));
	memcpy(a->v, h->v0, 32);
	a->src = h->dstage[h->cur];
	a->nst = h->fill / 32;
	a->v_dev = h->v_dev;
	a->out = h->dres;
	a->flags = flags | (h->folded ? NKFS_XXH_FROM_DEV : 0);
}

/* fold the staged chunk asynchronously; its buffer is reusable after ev */
static int xh_flush(struct xh *h)
{
	struct nkfs_xxh_args a;
	xh_args(h, &a, NKFS_XXH_TO_DEV);
	int err = nkfs_launch_xxh64_chain(&a, h->c->stream);
	if (err)
		return err;
	if (hipEventRecord(h->c->ev[h->cur], h->c->stream) != hipSuccess)
		return -EIO;
	h->inflight[h->cur] = 1;
	h->folded = 1;
	h->cur ^= 1;
	h->fill = 0;
	if (h->inflight[h->cur]) {  /* the fold two chunks back read this buffer */
		if (hipEventSynchronize(h->c->ev[h->cur]) != hipSuccess)
			return -EIO;
		h->inflight[h->cur] = 0;
	}
	return 0;
}

/* stage `bytes` (a multiple of 32) of whole stripes */
static int xh_stage(struct xh *h, const uint8_t *p, uint64_t bytes)
{
	while (bytes) {
		const uint64_t room = XH_CHUNK - h->fill;
		const uint64_t take = bytes < room ? bytes : room;
		memcpy(h->stage[h->cur] + h->fill, p, take);
		h->fill += (uint32_t)take;
		p += take;
		bytes -= take;
		if (h->fill == XH_CHUNK) {
			int err = xh_flush(h);
			if (err)
				return err;
		}
	}
	return 0;
}

/* ------------------------------------------- per-call service wave (opt-in)
 *
 * nkfs_percall_service(1) keeps one wave resident (k_xxh64_service) polling
 * a mailbox in coherent host memory: a message digested in one piece (no
 * earlier fold) is posted there instead of launched -- arguments, then the
 * request number -- and the host spins on the message's completion word as
 * before.  Requests are serialised by g_svc_lock (one box).  The wave leaves
 * after SVC_IDLE without requests (or SVC_LIFE in all); a request that finds
 * it gone, or that it never took, relaunches it once the service stream has
 * drained.
 *
 * nkfs_percall_service(2) (round 6): the request half of
 * the mailbox (seq, op, arguments, inline message) lives in uncached device
 * memory that the host writes directly through the PCIe BAR (a store
 * costs the host ~0.23 us, tools/bar_probe.c), so the wave's polls and
 * argument reads stay on the GPU; only the answer (digest, completion word,
 * taken, alive: the host-memory half) crosses PCIe to the host.  The host
 * keeps a shadow of seq, so it never reads device memory (a BAR read costs
 * ~1.2 us). */
#define SVC_IDLE 2000000ull      /* s_memrealtime ticks (100 MHz): 20 ms */
#define SVC_LIFE 1000000000ull   /* 10 s */
static pthread_mutex_t g_svc_lock = PTHREAD_MUTEX_INITIALIZER;
static struct nkfs_svc_box *g_svc_host, *g_svc_host_dev; /* coherent host memory: the answer half (both modes) */
static struct nkfs_svc_box *g_svc_bar;                   /* uncached device memory (mode 2), host-mapped */
static struct nkfs_svc_box *g_svc;                       /* the request half the host writes: host or BAR box */
static struct nkfs_svc_box *g_svc_in_dev;                /* the same, as the wave sees it */
static uint64_t g_svc_seq;                               /* the host's shadow of g_svc->seq */
static hipStream_t g_svc_stream;
static int g_svc_on, g_svc_mode, g_svc_device = -1, g_svc_exit_hooked;

/* publish the request number after the request (the BAR mapping is
 * write-combined: the fences keep the payload ahead of seq and push seq) */
static void svc_post_locked(uint64_t sq)
{
	__builtin_ia32_sfence();
	__atomic_store_n(&g_svc->seq, sq, __ATOMIC_RELEASE);
	__builtin_ia32_sfence();
	g_svc_seq = sq;
}

/* at exit: post a stop and give the wave a bounded time to leave (host
 * memory and the BAR only: no runtime calls while the process tears down) */
static void svc_atexit(void)
{
	if (!g_svc || !__atomic_load_n(&g_svc_host->alive, __ATOMIC_ACQUIRE))
		return;
	g_svc->op = NKFS_SVC_STOP;
	svc_post_locked(g_svc_seq + 1);
	struct timespec t0, t;
	clock_gettime(CLOCK_MONOTONIC, &t0);
	do {
		if (!__atomic_load_n(&g_svc_host->alive, __ATOMIC_ACQUIRE))
			return;
		clock_gettime(CLOCK_MONOTONIC, &t);
	} while ((t.tv_sec - t0.tv_sec) * 1000000000ll + (t.tv_nsec - t0.tv_nsec) < 100000000ll);
}

static int svc_launch_locked(void)
{
	__atomic_store_n(&g_svc_host->alive, 1, __ATOMIC_RELEASE);
	int err = nkfs_launch_xxh64_service(g_svc_in_dev, g_svc_host_dev, SVC_IDLE, SVC_LIFE, g_svc_stream);
	if (err)
		__atomic_store_n(&g_svc_host->alive, 0, __ATOMIC_RELEASE);
	return err;
}

/* stop a running wave (a stop uses a request number; the wave marks it
 * taken) and wait for its stream */
static int svc_stop_locked(void)
{
	if (!g_svc || !__atomic_load_n(&g_svc_host->alive, __ATOMIC_ACQUIRE))
		return 0;
	g_svc->op = NKFS_SVC_STOP;
	svc_post_locked(g_svc_seq + 1);
	return hipStreamSynchronize(g_svc_stream) != hipSuccess ? -EIO : 0;
}

int nkfs_percall_service(int on)
{
	if (on < 0 || on > 2)
		return -EINVAL;
	if (on && ensure_gpu())
		return -ENODEV;
	pthread_mutex_lock(&g_svc_lock);
	int err = 0;
	if (on && g_svc_on && on == g_svc_mode)
		goto out; /* already on in this mode: a live wave keeps its counters */
	if (!on || (g_svc_on && on != g_svc_mode)) {
		err = svc_stop_locked();
		__atomic_store_n(&g_svc_on, 0, __ATOMIC_RELEASE);
		if (!on || err)
			goto out;
	}
	if (!g_svc_host) {
		void *p = NULL, *dp = NULL;
		if (hipHostMalloc(&p, sizeof(*g_svc_host), hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
			err = -ENOMEM;
			goto out;
		}
		if (hipHostGetDevicePointer(&dp, p, 0) != hipSuccess ||
		    hipStreamCreateWithFlags(&g_svc_stream, hipStreamNonBlocking) != hipSuccess) {
			(void)hipHostFree(p);
			err = -EIO;
			goto out;
		}
		memset(p, 0, sizeof(*g_svc_host));
		g_svc_host = p;
		g_svc_host_dev = dp;
		(void)hipGetDevice(&g_svc_device);
		if (!g_svc_exit_hooked) {
			g_svc_exit_hooked = 1;
			atexit(svc_atexit);
		}
	}
	if (on == 2 && !g_svc_bar) {
		void *d = NULL;
		/* uncached: the wave's loads of the request never hit a line an
		 * earlier request left in its L2 (the host's BAR writes go around it) */
		if (hipExtMallocWithFlags(&d, sizeof(*g_svc_bar), hipDeviceMallocUncached) != hipSuccess ||
		    hipMemset(d, 0, sizeof(*g_svc_bar)) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
			(void)hipGetLastError();
			if (d)
				(void)hipFree(d);
			err = -ENOMEM;
			goto out;
		}
		g_svc_bar = d;
	}
	/* a fresh pair of counters for the chosen box: the request number and
	 * the taken mark start at 0 together (the wave starts from taken) */
	g_svc = on == 2 ? g_svc_bar : g_svc_host;
	g_svc_in_dev = on == 2 ? g_svc_bar : g_svc_host_dev;
	g_svc->seq = 0;
	__builtin_ia32_sfence();
	__atomic_store_n(&g_svc_host->taken, 0, __ATOMIC_RELEASE);
	g_svc_seq = 0;
	g_svc_mode = on;
	__atomic_store_n(&g_svc_on, 1, __ATOMIC_RELEASE);
out:
	pthread_mutex_unlock(&g_svc_lock);
	return err;
}

/* Run one message on the service wave and wait for its completion word;
 * -ENOSYS when the service is off (or on another device): launch instead. */
/* NKFS_SVC_TRACE=1: per-request phase times of the service path, printed
 * at exit (post -> the wave took the request -> completion word seen) */
static int g_svc_trace = -1;
static double g_tr_take, g_tr_done;
static uint64_t g_tr_n;

static double mono_us(void)
{
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static void svc_trace_report(void)
{
	if (g_tr_n)
		fprintf(stderr, "nkfs svc trace: %llu requests, post->taken %.2f us, taken->done %.2f us (means)\n",
			(unsigned long long)g_tr_n, g_tr_take / g_tr_n, g_tr_done / g_tr_n);
}

static int svc_run(const struct nkfs_xxh_args *a, const uint8_t *hsrc, volatile uint64_t *res)
{
	if (!__atomic_load_n(&g_svc_on, __ATOMIC_ACQUIRE))
		return -ENOSYS;
	int dev = -1;
	(void)hipGetDevice(&dev);
	pthread_mutex_lock(&g_svc_lock);
	if (!g_svc_on || dev != g_svc_device) {
		pthread_mutex_unlock(&g_svc_lock);
		return -ENOSYS;
	}
	int err = 0;
	/* the request is complete in the box before its number is published and
	 * before any (re)launch, so a wave never reads half-written arguments */
	struct nkfs_xxh_args ar = *a;
	/* a message of at most 1 KiB of stripes travels inline: the wave reads
	 * it in the same round trip as the arguments */
	if (a->nst * 32 <= NKFS_SVC_INL) {
		memcpy(g_svc->inl, hsrc, a->nst * 32);
		ar.src = g_svc_in_dev->inl;
		g_svc->op = NKFS_SVC_XXH_INL;
	} else {
		g_svc->op = NKFS_SVC_XXH;
	}
	g_svc->args = ar;
	const uint64_t sq = g_svc_seq + 1;
	if (g_svc_trace < 0) {
		g_svc_trace = getenv("NKFS_SVC_TRACE") != NULL;
		if (g_svc_trace)
			atexit(svc_trace_report);
	}
	const double t0 = g_svc_trace ? mono_us() : 0;
	double t1 = 0;
	svc_post_locked(sq);
	if (!__atomic_load_n(&g_svc_host->alive, __ATOMIC_ACQUIRE) && hipStreamQuery(g_svc_stream) == hipSuccess &&
	    (err = svc_launch_locked()))
		goto out;
	for (uint64_t spin = 0; __atomic_load_n(&res[1], __ATOMIC_ACQUIRE) != a->flag; spin++) {
		if (g_svc_trace && !t1 && __atomic_load_n(&g_svc_host->taken, __ATOMIC_ACQUIRE) == sq)
			t1 = mono_us();
		if ((spin & 0xFFF) == 0xFFF) {
			/* the service stream's own status, whether or not the wave took
			 * the request (a wave that faults or stalls after
			 * taking it must not spin the caller forever) */
			hipError_t q = hipStreamQuery(g_svc_stream);
			if (q != hipSuccess && q != hipErrorNotReady) {
				err = -EIO;
				goto out;
			}
			if (q == hipSuccess && __atomic_load_n(&res[1], __ATOMIC_ACQUIRE) != a->flag) {
				/* the wave is gone: it left before taking the request
				 * (relaunch), or took it and never finished (error) */
				if (__atomic_load_n(&g_svc_host->taken, __ATOMIC_ACQUIRE) == sq) {
					err = -EIO;
					goto out;
				}
				if ((err = svc_launch_locked()))
					goto out;
			}
		}
		__builtin_ia32_pause();
	}
	if (g_svc_trace) {
		const double t2 = mono_us();
		if (!t1)
			t1 = t2;
		g_tr_take += t1 - t0;
		g_tr_done += t2 - t1;
		g_tr_n++;
	}
out:
	pthread_mutex_unlock(&g_svc_lock);
	return err;
}

/* Launch the last fold with `flags` (EMIT / FINISH) and wait for its
 * completion word: a spin on pinned memory, with the stream's own status
 * checked now and then so a failed launch cannot spin forever. */
static int xh_complete(struct xh *h, uint32_t flags, const struct xstate *s, uint64_t *digest, uint64_t v[4])
{
	struct nkfs_xxh_args a;
	xh_args(h, &a, flags);
	if (s) {
		a.total_len = s->total_len;
		a.seed = s->seed;
		a.tail_len = s->memsize;
		memcpy(a.tail, s->mem64, s->memsize);
	}
	volatile uint64_t *res = (volatile uint64_t *)h->res;
	a.flag = ++h->c->seq | (1ull << 63);
	res[1] = 0;
	/* a message in one piece may go to the resident service wave */
	int err = h->folded ? -ENOSYS : svc_run(&a, h->stage[h->cur], res);
	if (err != -ENOSYS) {
		if (err)
			return err;
		goto done;
	}
	err = nkfs_launch_xxh64_chain(&a, h->c->stream);
	if (err)
		return err;
	for (uint64_t spin = 0; __atomic_load_n(&res[1], __ATOMIC_ACQUIRE) != a.flag; spin++) {
		if ((spin & 0xFFFF) == 0xFFFF) {
			hipError_t q = hipStreamQuery(h->c->stream);
			if (q != hipSuccess && q != hipErrorNotReady)
				return -EIO;
			if (q == hipSuccess && __atomic_load_n(&res[1], __ATOMIC_ACQUIRE) != a.flag)
				return -EIO; /* the stream drained without the word */
		}
		__builtin_ia32_pause();
	}
done:
	if (digest)
		*digest = res[0];
	if (v)
		for (int i = 0; i < 4; i++)
			v[i] = res[2 + i];
	return 0;
}

/* ------------------------------------------------------- pending slots */

/* At most NSLOT messages are pending on the GPU at once (each holds a
 * per-call context: a stream and 512 KiB of pinned staging); beyond that an
 * update folds synchronously (one round trip), so a burst of states -- or
 * states abandoned while pending (never digested, reset or freed), whose
 * slot stays taken -- cannot pin more than NSLOT contexts. */
#define NSLOT 64
#define PEND_MAGIC 0xC5A10000u
#define PEND_POISON (PEND_MAGIC | 0xFFFFu) /* a failed update: every later update / digest fails */

struct xslot {
	uint64_t token;
	int used;
	pthread_mutex_t mu; /* complete-and-free of this slot (concurrent digests of one state) */
	struct xh h;
};
static struct xslot g_slot[NSLOT] = { [0 ... NSLOT - 1] = { .mu = PTHREAD_MUTEX_INITIALIZER } };
static pthread_mutex_t g_slot_lock = PTHREAD_MUTEX_INITIALIZER;
static uint64_t g_token = 0x6E6B38465A5A0001ull;

/* the slot of a pending state, NULL if none; *stale = the state claims one
 * that is gone (a byte copy of a pending state that was digested) */
static struct xslot *slot_of(const struct xstate *s, int *stale)
{
	*stale = 0;
	const uint32_t pend = __atomic_load_n(&s->pend, __ATOMIC_ACQUIRE);
	if ((pend & 0xFFFF0000u) != PEND_MAGIC)
		return NULL;
	const uint32_t i = pend & 0xFFFFu;
	struct xslot *sl = i < NSLOT ? &g_slot[i] : NULL;
	pthread_mutex_lock(&g_slot_lock);
	const int ok = sl && sl->used && sl->token == __atomic_load_n(&s->v[0], __ATOMIC_RELAXED);
	pthread_mutex_unlock(&g_slot_lock);
	if (!ok) {
		*stale = 1;
		return NULL;
	}
	return sl;
}

static struct xslot *slot_take(void)
{
	pthread_mutex_lock(&g_slot_lock);
	for (int i = 0; i < NSLOT; i++)
		if (!g_slot[i].used) {
			g_slot[i].used = 1;
			g_slot[i].token = g_token++;
			pthread_mutex_unlock(&g_slot_lock);
			return &g_slot[i];
		}
	pthread_mutex_unlock(&g_slot_lock);
	return NULL;
}

static void slot_free(struct xslot *sl)
{
	xh_end(&sl->h);
	pthread_mutex_lock(&g_slot_lock);
	sl->used = 0;
	sl->token = 0;
	pthread_mutex_unlock(&g_slot_lock);
}

/* ------------------------------------------------------------ the ABI */

XXH_errorcode XXH64_freeState(XXH64_state_t *state)
{
	if (state) {
		struct xstate *s = (struct xstate *)state;
		int stale;
		struct xslot *sl = slot_of(s, &stale);
		if (sl)
			slot_free(sl);
	}
	crt_free(state);
	return XXH_OK;
}

XXH_errorcode XXH64_reset(XXH64_state_t *state_in, unsigned long long seed)
{
	struct xstate *s = (struct xstate *)state_in;
	int stale;
	struct xslot *sl = slot_of(s, &stale);
	if (sl) /* a message abandoned mid-stream */
		slot_free(sl);
	s->seed = seed;
	s->v[0] = seed + P1 + P2;
	s->v[1] = seed + P2;
	s->v[2] = seed;
	s->v[3] = seed - P1;
	s->total_len = 0;
	s->memsize = 0;
	s->pend = 0;
	return XXH_OK;
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
	int stale;
	struct xslot *sl = slot_of(s, &stale);
	if (stale)
		return XXH_ERROR;
	struct xh local, *h;
	if (sl) {
		h = &sl->h;
	} else {
		sl = slot_take();
		h = sl ? &sl->h : &local; /* no slot free: fold synchronously */
		if (xh_begin(h, s->v)) {
			if (sl)
				slot_free(sl);
			return XXH_ERROR; /* nothing of the state changed yet */
		}
		if (sl) {
			s->v[0] = sl->token;
			s->pend = PEND_MAGIC | (uint32_t)(sl - g_slot);
		}
	}
	int err = 0;
	if (s->memsize) {
		const size_t fill = 32 - s->memsize;
		memcpy((uint8_t *)s->mem64 + s->memsize, p, fill);
		p += fill;
		len -= fill;
		s->total_len += fill;
		s->memsize = 0;
		err = xh_stage(h, (const uint8_t *)s->mem64, 32);
	}
	const uint64_t nst = len / 32;
	if (!err && nst)
		err = xh_stage(h, p, nst * 32);
	if (!err && h == &local) {
		uint64_t v[4];
		err = xh_complete(h, NKFS_XXH_EMIT, NULL, NULL, v);
		if (!err)
			memcpy(s->v, v, 32);
	}
	if (h == &local)
		xh_end(h);
	if (err) {
		/* part of the input may already be folded or consumed from mem64:
		 * the state no longer describes any prefix of the input, so poison
		 * it -- every later update returns XXH_ERROR and a digest traps
		 * (as CRT_BUG) instead of returning a wrong sum; reset clears it */
		if (h != &local)
			slot_free(sl);
		__atomic_store_n(&s->pend, PEND_POISON, __ATOMIC_RELEASE);
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

/* returns 0 and fills *out, or a negative errno.  A pending message is
 * completed and its slot freed under the slot's mutex, and the state is
 * written back (accumulators, pend = 0) before the mutex is released: a
 * second digest of the same state (the reference's digest is read-only, so
 * callers may digest one state from two threads) then finds it no longer
 * pending and finishes from the written-back accumulators. */
static int finish(struct xstate *s, uint64_t *out)
{
	for (;;) {
		const uint32_t pend = __atomic_load_n(&s->pend, __ATOMIC_ACQUIRE);
		if (pend == PEND_POISON)
			return -EIO;
		if ((pend & 0xFFFF0000u) != PEND_MAGIC) {
			/* nothing on the GPU: merge + tail + avalanche in one launch */
			struct xh h;
			uint64_t v0[4];
			memcpy(v0, s->v, 32);
			int err = xh_begin(&h, v0);
			if (!err)
				err = xh_complete(&h, NKFS_XXH_FINISH, s, out, NULL);
			xh_end(&h);
			return err;
		}
		const uint32_t i = pend & 0xFFFFu;
		if (i >= NSLOT)
			return -EINVAL;
		struct xslot *sl = &g_slot[i];
		/* everything below under the slot's mutex: a concurrent digest that
		 * completes this message writes the accumulators into s->v and then
		 * clears s->pend while holding it, so the pair is never seen half
		 * written (pend still set, v[0] no longer the token) */
		pthread_mutex_lock(&sl->mu);
		if (__atomic_load_n(&s->pend, __ATOMIC_ACQUIRE) != pend) {
			pthread_mutex_unlock(&sl->mu); /* completed meanwhile: look again */
			continue;
		}
		pthread_mutex_lock(&g_slot_lock);
		const int mine = sl->used && sl->token == s->v[0];
		pthread_mutex_unlock(&g_slot_lock);
		if (!mine) { /* a byte copy of a state whose message is gone */
			pthread_mutex_unlock(&sl->mu);
			return -EINVAL;
		}
		uint64_t v[4];
		int err = xh_complete(&sl->h, NKFS_XXH_FINISH | NKFS_XXH_EMIT, s, out, v);
		if (!err) /* the state is now what the reference's is after the same updates */
			memcpy(s->v, v, 32);
		__atomic_store_n(&s->pend, err ? PEND_POISON : 0u, __ATOMIC_RELEASE);
		slot_free(sl);
		pthread_mutex_unlock(&sl->mu);
		return err;
	}
}

/* The reference returns a digest unconditionally; a GPU failure here has
 * no error channel, so it traps like CRT_BUG rather than return a wrong
 * checksum.  The accumulators of a pending message are written back into
 * the caller's state (it was writable: XXH64_update wrote it). */
unsigned long long XXH64_digest(const XXH64_state_t *state_in)
{
	uint64_t h;
	if (finish((struct xstate *)state_in, &h))
		__builtin_trap();
	return h;
}

unsigned long long XXH64(const void *input, size_t length, unsigned long long seed)
{
	XXH64_state_t st;
	memset(&st, 0, sizeof(st));
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
