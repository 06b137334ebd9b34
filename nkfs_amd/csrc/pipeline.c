/*
 * pipeline.c -- host-memory entry points: the path's real ends.  The
 * reference's PUT starts at the client socket, lands in core/upages.c page
 * buffers (an array of 4 KiB pages, core/upages.c:91-122) and ends on the
 * block device; its GET runs the other way (core/net.c:228-265,
 * client/lib/client.c:183-235).  Here a host batch --
 * contiguous blocks, a packed ragged batch or page lists -- streams through
 * the GPU in sub-batches:
 *
 *   encode:  blocks H2D -> fused encode + XXH64 -> parts and digests D2H
 *   decode:  parts H2D  -> K x K inverse + rebuild (+ part XXH64 verify)
 *            -> status D2H, then the blocks of the stripes that decoded D2H
 *
 * Each sub-batch rides one of three pooled per-call contexts (stream, device
 * scratch, pinned scratch), so the H2D of one sub-batch, the kernels of the
 * next and the D2H of a third overlap.  Page lists are gathered into /
 * scattered from pinned staging by the host (a page pointer is caller
 * memory the GPU never dereferences); contiguous caller buffers go straight
 * over DMA only when they are pinned allocations (hipHostMalloc, torch
 * pin_memory) or lie inside a range the caller registered once through
 * nkfs_host_register; any other (pageable) buffer is staged through the
 * context's pinned scratch by host copies, like a page list.  No DMA ever
 * targets pageable memory the library did not pin by allocation: both
 * host-path GPU faults of rounds 3 and 5 were DMA into pageable memory
 * through the runtime's SVM mapping (tools/pin_probe.c).
 * Only bytes the API defines as outputs are written back: part runs of
 * abutting stripes, blocks of stripes that decoded (gaps and failed stripes
 * keep the caller's bytes).
 *
 * With several device lanes (nkfs_gpu_set_devices) a batch is cut into
 * byte-balanced contiguous stripe ranges, one host thread and one device
 * lane each, no data exchanged between them (stripes are independent,
 * SURVEY.md §8(e)).
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

/* ------------------------------------------------------ pinned registry */

struct pin_ent {
	uintptr_t base;
	size_t bytes;
	int refs;
	int urefs; /* references held by nkfs_host_register (the rest: in-flight calls) */
	struct pin_ent *next;
};
static pthread_mutex_t g_pin_lock = PTHREAD_MUTEX_INITIALIZER;
static struct pin_ent *g_pins;
static uint64_t g_pin_calls;   /* registry references held by in-flight calls */
static int g_lanes_running;    /* host lane threads (atomics) */
static int g_copy_threads;     /* host copy threads (atomics) */

/* Is [p, p+bytes) inside ONE pinned allocation of the runtime
 * (hipHostMalloc, torch pin_memory)?  Only such memory is DMA'd without
 * staging.  Memory registered with hipHostRegister outside this library
 * reports no extent (hipMemGetAddressRange gives base NULL: it is a KFD SVM
 * range over pageable pages, tools/pin_probe.c E4) and is staged: the
 * library cannot know its lifetime, and DMA into pageable memory is what
 * faulted. */
static int runtime_pinned(const void *p, size_t bytes)
{
	hipPointerAttribute_t attr;
	if (hipPointerGetAttributes(&attr, p) != hipSuccess || attr.type != hipMemoryTypeHost) {
		(void)hipGetLastError();
		return 0;
	}
	void *base = NULL;
	size_t size = 0;
	const void *dp = attr.devicePointer ? attr.devicePointer : p;
	if (hipMemGetAddressRange(&base, &size, (void *)dp) != hipSuccess || !base || !size) {
		(void)hipGetLastError();
		return 0;
	}
	/* the range's offset inside the allocation, in the allocation's own VA */
	const uintptr_t off = (uintptr_t)dp - (uintptr_t)base;
	return off + bytes >= off && off + bytes <= size;
}

/* The registry holds only the caller's own registrations
 * (nkfs_host_register).  Which entry is [a, a+bytes) inside (NULL if none)?
 * *partial is set when it partly overlaps one.  Caller holds g_pin_lock. */
static struct pin_ent *pin_find(uintptr_t a, size_t bytes, int *partial)
{
	*partial = 0;
	for (struct pin_ent *e = g_pins; e; e = e->next) {
		if (a >= e->base && a + bytes <= e->base + e->bytes)
			return e;
		if (a < e->base + e->bytes && e->base < a + bytes)
			*partial = 1;
	}
	return NULL;
}

/* caller holds g_pin_lock */
static void pin_drop_locked(struct pin_ent *e)
{
	if (--e->refs == 0) {
		for (struct pin_ent **pp = &g_pins; *pp; pp = &(*pp)->next)
			if (*pp == e) {
				*pp = e->next;
				break;
			}
		const hipError_t he = hipHostUnregister((void *)e->base);
		if (he != hipSuccess) {
			(void)hipGetLastError();
			nkfs_hip_fail("hipHostUnregister", (int)he);
		}
		free(e);
	}
}

/* How a host call reaches the ranges it copies from / to ([p[i],
 * p[i]+bytes[i]), i < 2; NULL or empty ranges are skipped), decided in one
 * step under the registry lock:
 *  - inside an nkfs_host_register entry: a reference is taken (the owner's
 *    unregister cannot unpin it mid-call) and the range is DMA'd directly;
 *  - inside one pinned allocation of the runtime: DMA'd directly;
 *  - anything else (pageable memory, a range straddling a registration):
 *    staged through pinned scratch by host copies (direct[i] = 0).
 * Nothing is registered for a call.  held[i] = the entry to release. */
static void pin_take2(const void *const p[2], const size_t bytes[2], struct pin_ent *held[2], int direct[2])
{
	pthread_mutex_lock(&g_pin_lock);
	for (int i = 0; i < 2; i++) {
		held[i] = NULL;
		direct[i] = 0;
		if (!p[i] || !bytes[i])
			continue;
		int partial;
		struct pin_ent *in = pin_find((uintptr_t)p[i], bytes[i], &partial);
		if (in) {
			in->refs++;
			held[i] = in;
			direct[i] = 1;
		} else {
			direct[i] = runtime_pinned(p[i], bytes[i]);
		}
	}
	g_pin_calls += (held[0] != NULL) + (held[1] != NULL);
	pthread_mutex_unlock(&g_pin_lock);
}

static void pin_release2(struct pin_ent *held[2])
{
	pthread_mutex_lock(&g_pin_lock);
	for (int i = 0; i < 2; i++)
		if (held[i]) {
			g_pin_calls--;
			pin_drop_locked(held[i]);
			held[i] = NULL;
		}
	pthread_mutex_unlock(&g_pin_lock);
}

int nkfs_host_register(void *p, size_t bytes)
{
	if (!p || !bytes)
		return -EINVAL;
	const uintptr_t a = (uintptr_t)p;
	int rc = 0;
	pthread_mutex_lock(&g_pin_lock);
	int partial;
	struct pin_ent *in = pin_find(a, bytes, &partial);
	if (in) {
		in->refs++;
		in->urefs++; /* now also the caller's registration */
	} else if (partial) {
		rc = -EBUSY;
	} else if (runtime_pinned(p, bytes)) {
		rc = -EEXIST; /* pinned by its owner: nothing to hold */
	} else {
		struct pin_ent *e = malloc(sizeof(*e));
		hipError_t he = e ? hipHostRegister(p, bytes, hipHostRegisterPortable) : hipErrorOutOfMemory;
		if (!e) {
			rc = -ENOMEM;
		} else if (he != hipSuccess) {
			(void)hipGetLastError();
			free(e);
			rc = he == hipErrorHostMemoryAlreadyRegistered ? -EBUSY : nkfs_hip_fail("hipHostRegister", (int)he);
		} else {
			*e = (struct pin_ent){ a, bytes, 1, 1, g_pins };
			g_pins = e;
		}
	}
	pthread_mutex_unlock(&g_pin_lock);
	return rc;
}

int nkfs_host_unregister(void *p)
{
	/* lookup and release in one locked section: a concurrent drop cannot
	 * free the entry in between */
	pthread_mutex_lock(&g_pin_lock);
	struct pin_ent *e = g_pins;
	while (e && !(e->base == (uintptr_t)p && e->urefs))
		e = e->next;
	if (e) {
		e->urefs--;
		pin_drop_locked(e);
	}
	pthread_mutex_unlock(&g_pin_lock);
	return e ? 0 : -ENOENT;
}

/* ------------------------------------------------------- batch description */

enum { HP_ENC = 0, HP_DEC = 1 };

struct hp {
	int dir, n, k, n_slots, navail;
	uint32_t nstripes, max_block;
	/* uniform geometry (sizes == NULL) */
	uint32_t block_size;
	uint64_t block_pitch, part_pitch;
	/* ragged geometry */
	const uint32_t *sizes;
	const uint64_t *boff, *poff;
	/* block side: contiguous, or a page list */
	uint8_t *blocks;
	uint8_t *const *pages;
	const uint64_t *first_page;
	uint32_t page_size;
	/* part side: contiguous */
	uint8_t *parts;
	const uint8_t *ids, *avail;
	uint64_t *digests;
	const uint64_t *expect;
	uint64_t *badmask;
	int32_t *status;
	uint64_t chunk;
	/* pageable contiguous sides staged through pinned scratch (hp_run) */
	int stage_blk, stage_parts;
};

static uint32_t hp_B(const struct hp *h, uint32_t s) { return h->sizes ? h->sizes[s] : h->block_size; }

static int hp_slots(const struct hp *h) { return h->dir == HP_ENC ? h->n : h->n_slots; }

static uint64_t hp_ppitch(const struct hp *h, uint32_t s)
{
	return h->sizes ? nkfs_part_pitch(h->sizes[s], h->k) : h->part_pitch;
}

/* byte offsets of stripe s's block / part slots in the caller's buffers */
static uint64_t hp_bofs(const struct hp *h, uint32_t s)
{
	if (h->pages)
		return 0; /* page lists: no contiguous block side */
	return h->sizes ? h->boff[s] : (uint64_t)s * h->block_pitch;
}

static uint64_t hp_pofs(const struct hp *h, uint32_t s)
{
	return h->sizes ? h->poff[s] : (uint64_t)s * (uint64_t)hp_slots(h) * h->part_pitch;
}

static uint64_t hp_pspan(const struct hp *h, uint32_t s) { return (uint64_t)hp_slots(h) * hp_ppitch(h, s); }

static uint64_t align256(uint64_t v) { return (v + 255) & ~255ull; }

/* ------------------------------------------------------------ sub-batches */

#define NSTREAM_MAX 8 /* contexts (sub-batches in flight) per lane: struct nkfs_tune.host_depth */

/* Device / pinned scratch layout of one sub-batch of at most `cnt` stripes
 * (offsets into the context buffers). */
struct lay {
	uint64_t d_blk, d_parts, d_boff, d_poff, d_sz, d_ids, d_avail, d_dig, d_status, d_bad, d_work, d_scr, d_total;
	uint64_t h_boff, h_poff, h_sz, h_ids, h_avail, h_dig, h_status, h_bad, h_stage, h_pstage, h_total;
};

struct sub {
	uint32_t s0, s1;     /* stripes [s0, s1) */
	uint64_t blo, bhi;   /* caller block byte range (contiguous side) */
	uint64_t plo, phi;   /* caller part byte range */
	int live;            /* issued, not yet retired */
	int copied;          /* decode: block D2H issued */
	hipEvent_t ev;       /* decode: status ready */
};

struct lane {
	const struct hp *h;
	int dev;
	uint32_t s0, s1;
	int rc;
};

/* Next sub-batch starting at s0: consecutive stripes with at most
 * h->chunk bytes of blocks (at least one). */
static uint32_t sub_end(const struct hp *h, uint32_t s0, uint32_t lim)
{
	uint64_t bytes = hp_B(h, s0);
	uint32_t s1 = s0 + 1;
	while (s1 < lim && bytes + hp_B(h, s1) <= h->chunk)
		bytes += hp_B(h, s1++);
	return s1;
}

static void sub_ranges(const struct hp *h, struct sub *u)
{
	u->blo = hp_bofs(h, u->s0);
	u->plo = hp_pofs(h, u->s0);
	u->bhi = u->blo;
	u->phi = u->plo;
	for (uint32_t s = u->s0; s < u->s1; s++) {
		const uint64_t be = hp_bofs(h, s) + hp_B(h, s), pe = hp_pofs(h, s) + hp_pspan(h, s);
		u->bhi = be > u->bhi ? be : u->bhi;
		u->phi = pe > u->phi ? pe : u->phi;
	}
}

static int hp_paged(const struct hp *h) { return h->pages != NULL; }

static int ragged_ok(const uint32_t *sizes, const uint64_t *boff, const uint64_t *poff, uint32_t nstripes,
		     uint32_t max_block, int nsl, int k);

/* device bytes of the blocks of [s0, s1) */
static uint64_t dev_block_bytes(const struct hp *h, const struct sub *u)
{
	if (!hp_paged(h))
		return u->bhi - u->blo;
	uint64_t t = 0;
	for (uint32_t s = u->s0; s < u->s1; s++)
		t += align256(hp_B(h, s));
	return t;
}

static void layout(const struct hp *h, uint32_t cnt, uint64_t blk_bytes, uint64_t part_bytes, uint64_t scr_bytes,
		   struct lay *L)
{
	const uint64_t nsl = (uint64_t)hp_slots(h);
	uint64_t o = 0;
	L->d_blk = o;
	o += align256(blk_bytes);
	L->d_parts = o;
	o += align256(part_bytes);
	L->d_boff = o;
	o += align256(cnt * 8ull);
	L->d_poff = o;
	o += align256(cnt * 8ull);
	L->d_sz = o;
	o += align256(cnt * 4ull);
	L->d_ids = o;
	o += align256(cnt * nsl);
	L->d_avail = o;
	o += align256(cnt * (uint64_t)(h->navail > 0 ? h->navail : 1));
	L->d_dig = o;
	o += align256(cnt * nsl * 8);
	L->d_status = o;
	o += align256(cnt * 4ull);
	L->d_bad = o;
	o += align256(cnt * 8ull);
	L->d_work = o;
	o += align256(nkfs_decode_work_bytes(cnt, h->k));
	L->d_scr = o;
	o += align256(scr_bytes);
	L->d_total = o;

	o = 0;
	L->h_boff = o;
	o += align256(cnt * 8ull);
	L->h_poff = o;
	o += align256(cnt * 8ull);
	L->h_sz = o;
	o += align256(cnt * 4ull);
	L->h_ids = o;
	o += align256(cnt * nsl);
	L->h_avail = o;
	o += align256(cnt * (uint64_t)(h->navail > 0 ? h->navail : 1));
	L->h_dig = o;
	o += align256(cnt * nsl * 8);
	L->h_status = o;
	o += align256(cnt * 4ull);
	L->h_bad = o;
	o += align256(cnt * 8ull);
	L->h_stage = o; /* blocks: gathered pages or a staged pageable range */
	o += hp_paged(h) || h->stage_blk ? align256(blk_bytes) : 0;
	L->h_pstage = o; /* parts: a staged pageable range */
	o += h->stage_parts ? align256(part_bytes) : 0;
	L->h_total = o;
}

/* ------------------------------------------------------------ host copies */

/* Host copies between caller memory and pinned staging -- page gathers and
 * scatters, staged pageable ranges -- go through one list of (dst, src,
 * len) pieces run by a few threads: one memcpy stream tops out near 10
 * GB/s, below what PCIe moves.  Pieces are at most CP_PIECE bytes so a
 * single contiguous range spreads over the threads too. */
#define COPY_THREADS 4
#define CP_PIECE (1u << 20)

struct cp {
	uint8_t *dst;
	const uint8_t *src;
	size_t len;
};

struct cpl {
	struct cp *v;
	size_t n, cap;
	uint64_t bytes;
};

static void cpl_add(struct cpl *l, uint8_t *dst, const uint8_t *src, size_t len)
{
	while (len) {
		const size_t piece = len < CP_PIECE ? len : CP_PIECE;
		if (l->n == l->cap) {
			const size_t cap = l->cap ? 2 * l->cap : 256;
			struct cp *v = realloc(l->v, cap * sizeof(*v));
			if (!v) { /* no list: copy now, on this thread */
				memcpy(dst, src, len);
				return;
			}
			l->v = v;
			l->cap = cap;
		}
		l->v[l->n++] = (struct cp){ dst, src, piece };
		l->bytes += piece;
		dst += piece;
		src += piece;
		len -= piece;
	}
}

struct cpj {
	const struct cp *v;
	size_t a, b;
};

static void *cpj_run(void *arg)
{
	const struct cpj *j = arg;
	for (size_t i = j->a; i < j->b; i++)
		memcpy(j->v[i].dst, j->v[i].src, j->v[i].len);
	return NULL;
}

/* Run the list (byte-balanced contiguous shares, COPY_THREADS threads from
 * 4 MiB on) and empty it; every thread is joined before this returns. */
static void cpl_run(struct cpl *l)
{
	int nt = l->bytes >= (4u << 20) ? COPY_THREADS : 1;
	if ((size_t)nt > l->n)
		nt = (int)l->n;
	if (nt < 1)
		nt = 1;
	struct cpj jb[COPY_THREADS];
	pthread_t th[COPY_THREADS];
	int started[COPY_THREADS] = { 0 };
	uint64_t acc = 0;
	size_t a = 0;
	for (int t = 0; t < nt; t++) {
		const uint64_t goal = l->bytes * (uint64_t)(t + 1) / (uint64_t)nt;
		size_t b = a;
		while (b < l->n && (t == nt - 1 || acc < goal || b == a))
			acc += l->v[b++].len;
		jb[t] = (struct cpj){ l->v, a, b };
		a = b;
	}
	for (int t = 1; t < nt; t++) {
		started[t] = pthread_create(&th[t], NULL, cpj_run, &jb[t]) == 0;
		if (started[t])
			__atomic_add_fetch(&g_copy_threads, 1, __ATOMIC_RELAXED);
	}
	cpj_run(&jb[0]);
	for (int t = 1; t < nt; t++) {
		if (started[t]) {
			pthread_join(th[t], NULL);
			__atomic_sub_fetch(&g_copy_threads, 1, __ATOMIC_RELAXED);
		} else {
			cpj_run(&jb[t]);
		}
	}
	l->n = 0;
	l->bytes = 0;
}

static void cpl_free(struct cpl *l)
{
	free(l->v);
	memset(l, 0, sizeof(*l));
}

/* Gather (to_pages 0) or scatter (1) the blocks of stripes [s0, s1) between
 * their page lists and the packed staging `buf` (block s at its packed
 * 256-byte-aligned offset), stripes with status[s - s0] == -EINVAL left
 * alone. */
static int pages_copy(const struct hp *h, uint32_t s0, uint32_t s1, uint8_t *buf, uint64_t cap,
		      const int32_t *status, int to_pages)
{
	struct cpl l = { 0 };
	uint64_t o = 0;
	const uint32_t P = h->page_size;
	for (uint32_t s = s0; s < s1; s++) {
		const uint32_t B = hp_B(h, s);
		if (o + B > cap || o + B < o) { /* the staging region (always checked) */
			cpl_free(&l);
			return -ERANGE;
		}
		if (!status || status[s - s0] != -EINVAL) {
			uint8_t *const *pg = h->pages + h->first_page[s];
			for (uint32_t off = 0, i = 0; off < B; off += P, i++) {
				const uint32_t len = B - off < P ? B - off : P;
				if (to_pages)
					cpl_add(&l, pg[i], buf + o + off, len);
				else
					cpl_add(&l, buf + o + off, pg[i], len);
			}
		}
		o += align256(B);
	}
	cpl_run(&l);
	cpl_free(&l);
	return 0;
}

/* One contiguous range between caller memory and staging (threaded). */
static void range_copy(uint8_t *dst, const uint8_t *src, uint64_t len)
{
	struct cpl l = { 0 };
	cpl_add(&l, dst, src, len);
	cpl_run(&l);
	cpl_free(&l);
}

/* Sub-batch u's metadata into the pinned scratch `hb` (layout L): ids
 * (+ survivor lists and expected digests for a verifying decode) and, for
 * ragged batches, the block / part offsets shifted so that they land in
 * this context's device buffers, and the sizes.  [*lo, *hi) = the host range
 * the one metadata H2D copies (its device image starts at d_boff + (*lo -
 * h_boff): the two layouts list these regions in the same order). */
static void fill_meta(const struct hp *h, const struct sub *u, const struct lay *L, uint8_t *hb, uint64_t *lo,
		      uint64_t *hi)
{
	const uint32_t cnt = u->s1 - u->s0;
	const int nsl = hp_slots(h);
	memcpy(hb + L->h_ids, h->ids + (uint64_t)u->s0 * nsl, (size_t)cnt * nsl);
	uint64_t meta_lo = L->h_ids, meta_hi = L->h_ids + (uint64_t)cnt * nsl;
	if (h->dir == HP_DEC) {
		memcpy(hb + L->h_avail, h->avail + (uint64_t)u->s0 * h->navail, (size_t)cnt * h->navail);
		meta_hi = L->h_avail + (uint64_t)cnt * h->navail;
		if (h->expect) {
			memcpy(hb + L->h_dig, h->expect + (uint64_t)u->s0 * nsl, (size_t)cnt * nsl * 8);
			meta_hi = L->h_dig + (uint64_t)cnt * nsl * 8;
		}
	}
	if (h->sizes) {
		uint64_t *bo = (uint64_t *)(hb + L->h_boff), *po = (uint64_t *)(hb + L->h_poff);
		uint32_t *sz = (uint32_t *)(hb + L->h_sz);
		uint64_t packed = 0;
		for (uint32_t s = u->s0; s < u->s1; s++) {
			const uint32_t B = hp_B(h, s);
			if (hp_paged(h)) {
				bo[s - u->s0] = packed;
				packed += align256(B);
			} else {
				bo[s - u->s0] = h->boff[s] - u->blo;
			}
			po[s - u->s0] = h->poff[s] - u->plo;
			sz[s - u->s0] = B;
		}
		meta_lo = L->h_boff;
	}
	*lo = meta_lo;
	*hi = meta_hi;
}

/* Device scratch the launchers take for sub-batch u (ragged: size order +
 * slice map, nkfs_ragged_scratch_bytes; uniform batches need none). */
static uint64_t sub_scratch(const struct hp *h, const struct sub *u)
{
	if (!h->sizes)
		return 0;
	uint64_t units = 0;
	for (uint32_t s = u->s0; s < u->s1; s++)
		units += ((uint64_t)nkfs_part_size(hp_B(h, s), h->k) + 1023) / 1024;
	return nkfs_ragged_scratch_bytes(u->s1 - u->s0, units);
}

#define HIPGO(call, what)                                              \
	do {                                                           \
		hipError_t e_ = (call);                                \
		if (e_ != hipSuccess) {                                \
			rc = nkfs_hip_fail(what, (int)e_);             \
			goto out;                                      \
		}                                                      \
	} while (0)

struct ctxs {
	struct nkfs_ctx *c;
	uint8_t *d, *hb;
	struct lay L;
	struct sub u;
};

/* Issue sub-batch u on context x: metadata, H2D, kernels, and for encode
 * the D2H of parts and digests; for decode the status D2H + event. */
static int issue(const struct hp *h, struct ctxs *x)
{
	int rc = 0;
	const struct sub *u = &x->u;
	const uint32_t cnt = u->s1 - u->s0;
	const struct lay *L = &x->L;
	hipStream_t st = x->c->stream;
	uint8_t *d = x->d, *hb = x->hb;
	const int nsl = hp_slots(h);
	const int paged = hp_paged(h);

	/* metadata into pinned scratch: ids (+ survivor lists), ragged offsets */
	uint64_t meta_lo, meta_hi;
	fill_meta(h, u, L, hb, &meta_lo, &meta_hi);
	HIPGO(hipMemcpyAsync(d + L->d_boff + (meta_lo - L->h_boff), hb + meta_lo, meta_hi - meta_lo,
			     hipMemcpyHostToDevice, st),
	      "H2D (metadata)");

	/* payload in */
	if (h->dir == HP_ENC) {
		if (paged) {
			if ((rc = pages_copy(h, u->s0, u->s1, hb + L->h_stage, L->h_pstage - L->h_stage, NULL, 0)))
				goto out;
			uint64_t o = 0;
			for (uint32_t s = u->s0; s < u->s1; s++)
				o += align256(hp_B(h, s));
			HIPGO(hipMemcpyAsync(d + L->d_blk, hb + L->h_stage, o, hipMemcpyHostToDevice, st),
			      "H2D (gathered pages)");
		} else {
			const uint8_t *src = h->blocks + u->blo;
			if (h->stage_blk) { /* pageable: through pinned staging */
				range_copy(hb + L->h_stage, src, u->bhi - u->blo);
				src = hb + L->h_stage;
			}
			HIPGO(hipMemcpyAsync(d + L->d_blk, src, u->bhi - u->blo, hipMemcpyHostToDevice, st), "H2D (blocks)");
		}
	} else {
		const uint8_t *src = h->parts + u->plo;
		if (h->stage_parts) {
			range_copy(hb + L->h_pstage, src, u->phi - u->plo);
			src = hb + L->h_pstage;
		}
		HIPGO(hipMemcpyAsync(d + L->d_parts, src, u->phi - u->plo, hipMemcpyHostToDevice, st), "H2D (parts)");
	}

	/* kernels (bases shifted so that the caller-relative offsets land in
	 * this context's buffers) */
	const uint64_t dbp = paged ? align256(h->block_size) : h->block_pitch;
	struct nkfs_geom g;
	memset(&g, 0, sizeof(g));
	g.n = nsl;
	g.k = h->k;
	g.nstripes = cnt;
	g.blocks = d + L->d_blk;
	g.parts = d + L->d_parts;
	g.blocks_bytes = L->d_parts - L->d_blk;
	g.parts_bytes = L->d_boff - L->d_parts;
	if (L->d_total > L->d_scr) {
		g.scratch = d + L->d_scr;
		g.scratch_bytes = L->d_total - L->d_scr;
	}
	if (h->sizes) {
		g.block_size = h->max_block;
		g.block_off = (const uint64_t *)(d + L->d_boff);
		g.block_sizes = (const uint32_t *)(d + L->d_sz);
		g.part_off = (const uint64_t *)(d + L->d_poff);
	} else {
		g.block_size = h->block_size;
		g.block_pitch = dbp;
		g.part_pitch = h->part_pitch;
	}
	const void *gf = nkfs_gf_on(x->c->dev);
	if (!gf) {
		rc = -ENODEV;
		goto out;
	}
	if (h->dir == HP_ENC) {
		if ((rc = nkfs_launch_encode(&g, d + L->d_ids, h->digests ? (uint64_t *)(d + L->d_dig) : NULL, gf, st)))
			goto out;
		/* parts: runs of abutting stripes only (gaps keep the caller's bytes) */
		for (uint32_t s = u->s0; s < u->s1;) {
			uint64_t lo = hp_pofs(h, s), hi = lo + hp_pspan(h, s);
			uint32_t e = s + 1;
			while (e < u->s1 && hp_pofs(h, e) == hi)
				hi += hp_pspan(h, e++);
			uint8_t *dst = h->stage_parts ? hb + L->h_pstage + (lo - u->plo) : h->parts + lo;
			HIPGO(hipMemcpyAsync(dst, d + L->d_parts + (lo - u->plo), hi - lo, hipMemcpyDeviceToHost, st),
			      "D2H (parts)");
			s = e;
		}
		if (h->digests)
			HIPGO(hipMemcpyAsync(hb + L->h_dig, d + L->d_dig, (size_t)cnt * nsl * 8, hipMemcpyDeviceToHost, st),
			      "D2H (digests)");
	} else {
		rc = h->expect ? nkfs_launch_decode(&g, nsl, d + L->d_ids, d + L->d_avail, h->navail, d + L->d_work,
						    (int32_t *)(d + L->d_status), gf, st,
						    (const uint64_t *)(d + L->d_dig), (uint64_t *)(d + L->d_bad))
			       : nkfs_launch_decode(&g, nsl, d + L->d_ids, d + L->d_avail, h->navail, d + L->d_work,
						    (int32_t *)(d + L->d_status), gf, st, NULL, NULL);
		if (rc)
			goto out;
		HIPGO(hipMemcpyAsync(hb + L->h_status, d + L->d_status, (size_t)cnt * 4, hipMemcpyDeviceToHost, st),
		      "D2H (status)");
		if (h->badmask)
			HIPGO(hipMemcpyAsync(hb + L->h_bad, d + L->d_bad, (size_t)cnt * 8, hipMemcpyDeviceToHost, st),
			      "D2H (badmask)");
		HIPGO(hipEventRecord(x->u.ev, st), "event record");
	}
out:
	return rc;
}

/* Decode, second stage: once the status is on the host, copy back the
 * blocks of the stripes that decoded (a stripe with fewer than k distinct
 * ids keeps the caller's bytes, as nk8_assemble_block leaves its block). */
static int copy_blocks(const struct hp *h, struct ctxs *x)
{
	int rc = 0;
	const struct sub *u = &x->u;
	hipStream_t st = x->c->stream;
	HIPGO(hipEventSynchronize(u->ev), "status wait");
	const int32_t *stv = (const int32_t *)(x->hb + x->L.h_status);
	const int paged = hp_paged(h);
	uint64_t packed = 0;
	for (uint32_t s = u->s0; s < u->s1;) {
		if (stv[s - u->s0] == -EINVAL) {
			packed += align256(hp_B(h, s));
			s++;
			continue;
		}
		if (paged) {
			/* whole sub-batch staging is contiguous: copy runs of good stripes */
			uint64_t lo = packed, hi = packed + align256(hp_B(h, s));
			uint32_t e = s + 1;
			while (e < u->s1 && stv[e - u->s0] != -EINVAL)
				hi += align256(hp_B(h, e++));
			HIPGO(hipMemcpyAsync(x->hb + x->L.h_stage + lo, x->d + x->L.d_blk + lo, hi - lo,
					     hipMemcpyDeviceToHost, st),
			      "D2H (blocks to staging)");
			packed = hi;
			s = e;
		} else if (!h->sizes && h->block_pitch != h->block_size) {
			uint32_t e = s + 1;
			while (e < u->s1 && stv[e - u->s0] != -EINVAL)
				e++;
			const uint64_t lo = hp_bofs(h, s);
			uint8_t *dst = h->stage_blk ? x->hb + x->L.h_stage + (lo - u->blo) : h->blocks + lo;
			HIPGO(hipMemcpy2DAsync(dst, h->block_pitch, x->d + x->L.d_blk + (lo - u->blo), h->block_pitch,
					       h->block_size, e - s, hipMemcpyDeviceToHost, st),
			      "D2H (blocks, pitched)");
			s = e;
		} else {
			uint64_t lo = hp_bofs(h, s), hi = lo + hp_B(h, s);
			uint32_t e = s + 1;
			while (e < u->s1 && stv[e - u->s0] != -EINVAL && hp_bofs(h, e) == hi)
				hi += hp_B(h, e++);
			uint8_t *dst = h->stage_blk ? x->hb + x->L.h_stage + (lo - u->blo) : h->blocks + lo;
			HIPGO(hipMemcpyAsync(dst, x->d + x->L.d_blk + (lo - u->blo), hi - lo, hipMemcpyDeviceToHost, st),
			      "D2H (blocks)");
			s = e;
		}
	}
	x->u.copied = 1;
out:
	return rc;
}

/* Last stage: wait for the context's stream, then -- only for a sub-batch
 * whose stages all succeeded (`publish`; a decode's blocks copied back) --
 * hand the small outputs to the caller (digests / status / badmask) and
 * scatter decoded pages.  After a failure the staging may hold an earlier
 * sub-batch's bytes, so nothing of it reaches the caller. */
static int retire(const struct hp *h, struct ctxs *x, int publish)
{
	int rc = 0;
	const struct sub *u = &x->u;
	const uint32_t cnt = u->s1 - u->s0;
	const int nsl = hp_slots(h);
	HIPGO(hipStreamSynchronize(x->c->stream), "pipeline sync");
	if (!publish || (h->dir == HP_DEC && !u->copied))
		goto out;
	if (h->dir == HP_ENC) {
		if (h->digests)
			memcpy(h->digests + (uint64_t)u->s0 * nsl, x->hb + x->L.h_dig, (size_t)cnt * nsl * 8);
		if (h->stage_parts) { /* the part runs issue() copied into staging */
			struct cpl l = { 0 };
			for (uint32_t s = u->s0; s < u->s1;) {
				uint64_t lo = hp_pofs(h, s), hi = lo + hp_pspan(h, s);
				uint32_t e = s + 1;
				while (e < u->s1 && hp_pofs(h, e) == hi)
					hi += hp_pspan(h, e++);
				cpl_add(&l, h->parts + lo, x->hb + x->L.h_pstage + (lo - u->plo), hi - lo);
				s = e;
			}
			cpl_run(&l);
			cpl_free(&l);
		}
	} else {
		const int32_t *stv = (const int32_t *)(x->hb + x->L.h_status);
		if (h->status)
			memcpy(h->status + u->s0, stv, (size_t)cnt * 4);
		if (h->badmask)
			memcpy(h->badmask + u->s0, x->hb + x->L.h_bad, (size_t)cnt * 8);
		if (hp_paged(h)) {
			rc = pages_copy(h, u->s0, u->s1, x->hb + x->L.h_stage, x->L.h_pstage - x->L.h_stage, stv, 1);
		} else if (h->stage_blk) { /* the blocks of the stripes that decoded */
			struct cpl l = { 0 };
			for (uint32_t s = u->s0; s < u->s1; s++)
				if (stv[s - u->s0] != -EINVAL)
					cpl_add(&l, h->blocks + hp_bofs(h, s), x->hb + x->L.h_stage + (hp_bofs(h, s) - u->blo),
						hp_B(h, s));
			cpl_run(&l);
			cpl_free(&l);
		}
	}
out:
	x->u.live = 0;
	return rc;
}

/* One device lane: stripes [s0, s1) of the batch on device `dev`. */
static int run_lane(const struct hp *h, int dev, uint32_t s0, uint32_t s1)
{
	if (s0 >= s1)
		return 0;
	/* scratch sized for the largest sub-batch of this lane */
	uint64_t max_blk = 0, max_parts = 0, max_scr = 0;
	uint32_t max_cnt = 0;
	for (uint32_t s = s0; s < s1;) {
		struct sub u = { .s0 = s, .s1 = sub_end(h, s, s1) };
		sub_ranges(h, &u);
		const uint64_t bb = dev_block_bytes(h, &u), sb = sub_scratch(h, &u);
		max_blk = bb > max_blk ? bb : max_blk;
		max_parts = u.phi - u.plo > max_parts ? u.phi - u.plo : max_parts;
		max_cnt = u.s1 - u.s0 > max_cnt ? u.s1 - u.s0 : max_cnt;
		max_scr = sb > max_scr ? sb : max_scr;
		s = u.s1;
	}
	const int NSTREAM = nkfs_host_depth();
	struct ctxs xs[NSTREAM_MAX];
	memset(xs, 0, sizeof(xs));
	int rc = 0;
	for (int i = 0; i < NSTREAM; i++) {
		struct ctxs *x = &xs[i];
		layout(h, max_cnt, max_blk, max_parts, max_scr, &x->L);
		void *dv, *hv;
		if (!(x->c = nkfs_ctx_get_on(dev))) {
			rc = -ENOMEM;
			goto out;
		}
		if ((rc = nkfs_ctx_dev(x->c, x->L.d_total, &dv)) || (rc = nkfs_ctx_host(x->c, x->L.h_total, &hv)))
			goto out;
		x->d = dv;
		x->hb = hv;
		if (h->dir == HP_DEC && hipEventCreateWithFlags(&x->u.ev, hipEventDisableTiming) != hipSuccess) {
			x->u.ev = NULL;
			rc = -EIO;
			goto out;
		}
	}
	/* stages per context: issue -> (decode) copy_blocks -> retire, with up
	 * to three sub-batches in flight: sub-batch i is issued, i-1's blocks
	 * are copied back once its status is known, i-2 retires */
	struct ctxs *ring[NSTREAM_MAX] = {0};
	uint32_t it = 0;
	for (uint32_t s = s0; s < s1 && !rc; it++) {
		struct ctxs *x = &xs[it % NSTREAM];
		if (x->u.live && (rc = retire(h, x, 1)))
			break;
		hipEvent_t ev = x->u.ev;
		memset(&x->u, 0, sizeof(x->u));
		x->u.ev = ev;
		x->u.s0 = s;
		x->u.s1 = sub_end(h, s, s1);
		sub_ranges(h, &x->u);
		x->u.live = 1;
		if ((rc = issue(h, x)))
			break;
		ring[it % NSTREAM] = x;
		if (h->dir == HP_DEC && it >= 1) {
			struct ctxs *p = ring[(it - 1) % NSTREAM];
			if (p && p->u.live && !p->u.copied && (rc = copy_blocks(h, p)))
				break;
		}
		s = x->u.s1;
	}
	/* drain in issue order */
	for (uint32_t j = 0; j < (uint32_t)NSTREAM; j++) {
		struct ctxs *x = &xs[(it + j) % NSTREAM];
		if (!x->u.live)
			continue;
		int r = 0;
		if (!rc && h->dir == HP_DEC && !x->u.copied)
			r = copy_blocks(h, x);
		int r2 = retire(h, x, !rc && !r);
		if (!rc)
			rc = r ? r : r2;
	}
out:
	for (int i = 0; i < NSTREAM; i++) {
		if (xs[i].c) {
			if (xs[i].u.live)
				hipStreamSynchronize(xs[i].c->stream);
			nkfs_ctx_put(xs[i].c);
		}
		if (xs[i].u.ev)
			hipEventDestroy(xs[i].u.ev);
	}
	return rc;
}

static void *lane_main(void *arg)
{
	struct lane *l = arg;
	__atomic_add_fetch(&g_lanes_running, 1, __ATOMIC_RELAXED);
	l->rc = run_lane(l->h, l->dev, l->s0, l->s1);
	__atomic_sub_fetch(&g_lanes_running, 1, __ATOMIC_RELAXED);
	return NULL;
}

int nkfs_host_lane_plan(const int *devices, int ndev, int per_device, int *lanes, int max_lanes)
{
	if (!devices || !lanes || ndev < 1 || max_lanes < 1)
		return 0;
	if (per_device < 1)
		per_device = 1;
	/* device-interleaved rounds (filling device by device let
	 * the NKFS_MAX_DEVICES cap drop the trailing devices entirely) */
	int nl = 0;
	for (int j = 0; j < per_device; j++)
		for (int i = 0; i < ndev; i++) {
			if (nl == max_lanes)
				return nl;
			lanes[nl++] = devices[i];
		}
	return nl;
}

/* Pin the contiguous caller buffers, cut the batch over the device lanes
 * (byte-balanced contiguous stripe ranges) and run them. */
static int hp_run(struct hp *h)
{
	if (!h->chunk)
		h->chunk = 32ull << 20;
	uint64_t bend = 0, pend = 0, total = 0;
	for (uint32_t s = 0; s < h->nstripes; s++) {
		const uint64_t be = hp_bofs(h, s) + hp_B(h, s), pe = hp_pofs(h, s) + hp_pspan(h, s);
		bend = be > bend ? be : bend;
		pend = pe > pend ? pe : pend;
		total += hp_B(h, s);
	}
	struct pin_ent *held[2];
	int direct[2];
	const void *rp[2] = { hp_paged(h) ? NULL : h->blocks, h->parts };
	const size_t rb[2] = { bend, pend };
	pin_take2(rp, rb, held, direct);
	h->stage_blk = !hp_paged(h) && !direct[0];
	h->stage_parts = !direct[1];
	int rc = 0;
	/* struct nkfs_tune.host_lanes host threads per device: each lane keeps
	 * its own host_depth sub-batches in flight, so one host thread blocked
	 * on a stream never leaves the link idle */
	int dv[NKFS_MAX_DEVICES], lanes[NKFS_MAX_DEVICES];
	const int nd = nkfs_gpu_get_devices(dv, NKFS_MAX_DEVICES);
	int nl = nkfs_host_lane_plan(dv, nd, nkfs_host_lanes(), lanes, NKFS_MAX_DEVICES);
	if (nl > (int)h->nstripes)
		nl = (int)h->nstripes;
	if (nl <= 1) {
		rc = run_lane(h, lanes[0], 0, h->nstripes);
		/* the lane made its device current: hand the library's back */
		nkfs_use_device(nkfs_gpu_device());
	} else {
		struct lane L[NKFS_MAX_DEVICES];
		pthread_t th[NKFS_MAX_DEVICES];
		int started[NKFS_MAX_DEVICES] = {0};
		uint64_t acc = 0;
		uint32_t s = 0;
		for (int i = 0; i < nl; i++) {
			/* lane i ends where the running byte total passes (i+1)/nl */
			const uint64_t goal = total * (uint64_t)(i + 1) / (uint64_t)nl;
			uint32_t e = s;
			while (e < h->nstripes && (i == nl - 1 || acc + hp_B(h, e) <= goal || e == s)) {
				acc += hp_B(h, e);
				e++;
			}
			L[i] = (struct lane){ h, lanes[i], s, e, 0 };
			s = e;
		}
		for (int i = 1; i < nl; i++)
			started[i] = pthread_create(&th[i], NULL, lane_main, &L[i]) == 0;
		lane_main(&L[0]);
		for (int i = 1; i < nl; i++) {
			if (started[i])
				pthread_join(th[i], NULL);
			else
				lane_main(&L[i]); /* no thread: run it here */
		}
		for (int i = 0; i < nl && !rc; i++)
			rc = L[i].rc;
		nkfs_use_device(nkfs_gpu_device());
	}
	pin_release2(held);
	return rc;
}

int nkfs_host_state(uint64_t *out, int n)
{
	uint64_t v[5] = { 0 };
	pthread_mutex_lock(&g_pin_lock);
	for (struct pin_ent *e = g_pins; e; e = e->next)
		v[0]++;
	v[1] = g_pin_calls;
	pthread_mutex_unlock(&g_pin_lock);
	v[2] = (uint64_t)__atomic_load_n(&g_lanes_running, __ATOMIC_RELAXED);
	v[3] = (uint64_t)__atomic_load_n(&g_copy_threads, __ATOMIC_RELAXED);
	v[4] = nkfs_ctx_outstanding();
	if (!out || n < 0)
		return -EINVAL;
	for (int i = 0; i < n && i < 5; i++)
		out[i] = v[i];
	return 5;
}

/* ------------------------------------------------------------ plan check */

#define CHK(cond, ...)                                                         \
	do {                                                                   \
		if (!(cond)) {                                                 \
			if (msg && msg_len)                                    \
				snprintf(msg, msg_len, __VA_ARGS__);           \
			rc = -ERANGE;                                          \
			goto out;                                              \
		}                                                              \
	} while (0)

static int in_range(uint64_t lo, uint64_t len, uint64_t rlo, uint64_t rhi)
{
	return lo >= rlo && lo + len >= lo && lo + len <= rhi;
}

/* CPU replay of a ragged host call's plan (hp_run -> run_lane -> issue):
 * the same sub-batch cuts, layout and shifted offsets (fill_meta writes
 * them into a host copy of the pinned scratch), then every access the
 * kernels and copies of each sub-batch make is checked against the region
 * it must stay in: block reads up to the walk encoder's dword-rounded
 * num_records, part stores over the stripe's n_slots * pitch, the metadata
 * image, the launchers' scratch, the caller-side copy ranges.  Touches no
 * GPU (round-3 fault audit; tests/test_abi.py). */
int nkfs_pipeline_check(int decode, const uint64_t *block_off, const uint32_t *block_size, uint32_t max_block_size,
			uint32_t nstripes, int n_slots, int k, int navail, const uint64_t *part_off, uint32_t page_size,
			uint64_t chunk_bytes, char *msg, size_t msg_len)
{
	if (!block_size || !part_off || (!page_size && !block_off) || nkfs_bad_params(max_block_size, n_slots, k) ||
	    (decode && (navail < k || navail > n_slots)) ||
	    !ragged_ok(block_size, page_size ? NULL : block_off, part_off, nstripes, max_block_size, n_slots, k))
		return -EINVAL;
	uint64_t *first = NULL;
	uint8_t *ids = NULL, *avail = NULL, *hb = NULL;
	int rc = 0, subs = 0;
	first = calloc(nstripes ? nstripes : 1, sizeof(*first));
	ids = calloc((size_t)(nstripes ? nstripes : 1) * n_slots, 1);
	avail = calloc((size_t)(nstripes ? nstripes : 1) * (navail > 0 ? navail : 1), 1);
	if (!first || !ids || !avail) {
		rc = -ENOMEM;
		goto out;
	}
	struct hp h = { .dir = decode ? HP_DEC : HP_ENC, .n = n_slots, .k = k, .n_slots = decode ? n_slots : 0,
			.navail = decode ? navail : 0, .nstripes = nstripes, .max_block = max_block_size,
			.sizes = block_size, .boff = page_size ? NULL : block_off, .poff = part_off, .ids = ids,
			.avail = avail, .chunk = chunk_bytes ? chunk_bytes : 32ull << 20,
			/* pageable caller buffers: both sides staged (the default) */
			.stage_blk = page_size ? 0 : 1, .stage_parts = 1 };
	if (page_size) { /* page lists: only the packed staging matters here */
		h.pages = (uint8_t *const *)first; /* non-NULL marker, never dereferenced */
		h.first_page = first;
		h.page_size = page_size;
	}
	/* caller buffer extents (hp_run) */
	uint64_t bend = 0, pend = 0;
	for (uint32_t s = 0; s < nstripes; s++) {
		const uint64_t be = hp_bofs(&h, s) + hp_B(&h, s), pe = hp_pofs(&h, s) + hp_pspan(&h, s);
		bend = be > bend ? be : bend;
		pend = pe > pend ? pe : pend;
	}
	/* run_lane's scratch sizing */
	uint64_t max_blk = 0, max_parts = 0, max_scr = 0;
	uint32_t max_cnt = 0;
	for (uint32_t s = 0; s < nstripes;) {
		struct sub u = { .s0 = s, .s1 = sub_end(&h, s, nstripes) };
		sub_ranges(&h, &u);
		const uint64_t bb = dev_block_bytes(&h, &u), sb = sub_scratch(&h, &u);
		max_blk = bb > max_blk ? bb : max_blk;
		max_parts = u.phi - u.plo > max_parts ? u.phi - u.plo : max_parts;
		max_cnt = u.s1 - u.s0 > max_cnt ? u.s1 - u.s0 : max_cnt;
		max_scr = sb > max_scr ? sb : max_scr;
		s = u.s1;
	}
	struct lay L;
	layout(&h, max_cnt, max_blk, max_parts, max_scr, &L);
	CHK(L.d_blk < L.d_parts && L.d_parts <= L.d_boff && L.d_boff <= L.d_poff && L.d_poff <= L.d_sz &&
		    L.d_sz <= L.d_ids && L.d_ids <= L.d_avail && L.d_avail <= L.d_dig && L.d_dig <= L.d_status &&
		    L.d_status <= L.d_bad && L.d_bad <= L.d_work && L.d_work <= L.d_scr && L.d_scr <= L.d_total,
	    "device layout regions out of order");
	CHK(L.d_ids - L.d_boff == L.h_ids - L.h_boff && L.d_dig - L.d_boff == L.h_dig - L.h_boff,
	    "host and device metadata images differ");
	hb = calloc(L.h_total ? L.h_total : 1, 1);
	if (!hb) {
		rc = -ENOMEM;
		goto out;
	}
	for (uint32_t s = 0; s < nstripes; subs++) {
		struct sub u = { .s0 = s, .s1 = sub_end(&h, s, nstripes) };
		sub_ranges(&h, &u);
		const uint32_t cnt = u.s1 - u.s0;
		uint64_t lo, hi;
		fill_meta(&h, &u, &L, hb, &lo, &hi);
		CHK(in_range(L.d_boff + (lo - L.h_boff), hi - lo, L.d_boff, L.d_status), "sub-batch %d: metadata image", subs);
		if (!page_size) {
			CHK(in_range(u.blo, u.bhi - u.blo, 0, bend), "sub-batch %d: block H2D/D2H range", subs);
			CHK(u.bhi - u.blo <= L.d_parts - L.d_blk, "sub-batch %d: blocks exceed the device region", subs);
		}
		CHK(in_range(u.plo, u.phi - u.plo, 0, pend), "sub-batch %d: part copy range", subs);
		CHK(u.phi - u.plo <= L.d_boff - L.d_parts, "sub-batch %d: parts exceed the device region", subs);
		/* host staging: gathered pages / a staged block range, a staged part range */
		CHK(dev_block_bytes(&h, &u) <= L.h_pstage - L.h_stage, "sub-batch %d: block staging", subs);
		CHK(u.phi - u.plo <= L.h_total - L.h_pstage, "sub-batch %d: part staging", subs);
		CHK(sub_scratch(&h, &u) <= L.d_total - L.d_scr, "sub-batch %d: launcher scratch", subs);
		CHK((uint64_t)cnt * n_slots * 8 <= L.d_status - L.d_dig, "sub-batch %d: digest region", subs);
		CHK(nkfs_decode_work_bytes(cnt, k) <= L.d_scr - L.d_work, "sub-batch %d: decode workspace", subs);
		const uint64_t *bo = (const uint64_t *)(hb + L.h_boff), *po = (const uint64_t *)(hb + L.h_poff);
		const uint32_t *sz = (const uint32_t *)(hb + L.h_sz);
		for (uint32_t i = 0; i < cnt; i++) {
			const uint32_t B = sz[i];
			CHK(B == hp_B(&h, u.s0 + i), "stripe %u: size image", u.s0 + i);
			/* block side: reads up to the dword-rounded num_records of the
			 * walk encoder's buffer resource; decode writes [bo, bo + B) */
			CHK(in_range(bo[i], ((uint64_t)B + 3) & ~3ull, 0, L.d_parts - L.d_blk),
			    "stripe %u: block bytes [%llu, +%u) outside the device block region (%llu)", u.s0 + i,
			    (unsigned long long)bo[i], B, (unsigned long long)(L.d_parts - L.d_blk));
			CHK(in_range(po[i], (uint64_t)n_slots * nkfs_part_pitch(B, k), 0, L.d_boff - L.d_parts),
			    "stripe %u: parts [%llu, +%llu) outside the device part region", u.s0 + i,
			    (unsigned long long)po[i], (unsigned long long)((uint64_t)n_slots * nkfs_part_pitch(B, k)));
			CHK((po[i] & 15) == 0, "stripe %u: part base not 16-byte aligned", u.s0 + i);
		}
		s = u.s1;
	}
	if (msg && msg_len)
		snprintf(msg, msg_len, "ok: %d sub-batch(es), device %llu B per context", subs,
			 (unsigned long long)L.d_total);
out:
	free(hb);
	free(avail);
	free(ids);
	free(first);
	return rc;
}

/* ----------------------------------------------------------- entry points */

static int ragged_ok(const uint32_t *sizes, const uint64_t *boff, const uint64_t *poff, uint32_t nstripes,
		     uint32_t max_block, int nsl, int k)
{
	for (uint32_t s = 0; s < nstripes; s++) {
		if (!sizes[s] || sizes[s] > max_block)
			return 0;
		if (boff && s && boff[s] < boff[s - 1] + sizes[s - 1])
			return 0; /* blocks overlap or go backwards */
		if (s && poff[s] < poff[s - 1] + (uint64_t)nsl * nkfs_part_pitch(sizes[s - 1], k))
			return 0;
		if (poff[s] & 15)
			return 0;
	}
	return 1;
}

static int pages_ok(uint8_t *const *pages, uint32_t page_size, const uint64_t *first_page, uint32_t nstripes)
{
	if (!pages || !first_page || page_size < 8)
		return 0;
	(void)nstripes;
	return 1;
}

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
	struct hp h = { .dir = HP_ENC, .n = n, .k = k, .nstripes = nstripes, .max_block = block_size,
			.block_size = block_size, .block_pitch = nstripes > 1 ? block_pitch : block_size,
			.part_pitch = part_pitch, .blocks = (uint8_t *)h_blocks, .parts = h_parts, .ids = h_ids,
			.digests = h_digests, .chunk = chunk_bytes };
	return hp_run(&h);
}

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
	if (!h_blocks || !h_block_off || !h_block_size || !h_ids || !h_parts || !h_part_off ||
	    !ragged_ok(h_block_size, h_block_off, h_part_off, nstripes, max_block_size, n, k))
		return -EINVAL;
	struct hp h = { .dir = HP_ENC, .n = n, .k = k, .nstripes = nstripes, .max_block = max_block_size,
			.sizes = h_block_size, .boff = h_block_off, .poff = h_part_off, .blocks = (uint8_t *)h_blocks,
			.parts = h_parts, .ids = h_ids, .digests = h_digests, .chunk = chunk_bytes };
	return hp_run(&h);
}

int nkfs_nk8_encode_pages(const uint8_t *const *h_pages, uint32_t page_size, const uint64_t *h_first_page,
			  const uint32_t *h_block_size, uint32_t max_block_size, uint32_t nstripes, int n, int k,
			  const uint8_t *h_ids, uint8_t *h_parts, const uint64_t *h_part_off, uint64_t *h_digests,
			  uint64_t chunk_bytes)
{
	if (nkfs_bad_params(max_block_size, n, k))
		return -EINVAL;
	if (!nkfs_gpu_ready())
		return -EAGAIN;
	if (!nstripes)
		return 0;
	if (!h_block_size || !h_ids || !h_parts || !h_part_off ||
	    !pages_ok((uint8_t *const *)h_pages, page_size, h_first_page, nstripes) ||
	    !ragged_ok(h_block_size, NULL, h_part_off, nstripes, max_block_size, n, k))
		return -EINVAL;
	struct hp h = { .dir = HP_ENC, .n = n, .k = k, .nstripes = nstripes, .max_block = max_block_size,
			.sizes = h_block_size, .poff = h_part_off, .pages = (uint8_t *const *)h_pages,
			.first_page = h_first_page, .page_size = page_size, .parts = h_parts, .ids = h_ids,
			.digests = h_digests, .chunk = chunk_bytes };
	return hp_run(&h);
}

/* every offered slot must exist: the kernels index the stripe's id row
 * with it (a device-resident caller owns this precondition, nkfs_gpu.h) */
static int avail_ok(const uint8_t *avail, uint32_t nstripes, int navail, int n_slots)
{
	const uint64_t cnt = (uint64_t)nstripes * (uint64_t)navail;
	for (uint64_t i = 0; i < cnt; i++)
		if (avail[i] >= n_slots)
			return 0;
	return 1;
}

static int dec_args_ok(int n_slots, int navail, int k, uint32_t block_size, const uint8_t *ids, const uint8_t *avail,
		       uint32_t nstripes)
{
	return !nkfs_bad_params(block_size, navail, k) && n_slots >= 1 && n_slots <= 255 && ids && avail &&
	       avail_ok(avail, nstripes, navail, n_slots);
}

int nkfs_nk8_decode_host(const uint8_t *h_parts, uint64_t part_pitch, int n_slots, const uint8_t *h_ids,
			 const uint8_t *h_avail, int navail, int k, uint32_t block_size, uint8_t *h_blocks,
			 uint64_t block_pitch, uint32_t nstripes, int32_t *h_status, const uint64_t *h_expect,
			 uint64_t *h_badmask, uint64_t chunk_bytes)
{
	if (!dec_args_ok(n_slots, navail, k, block_size, h_ids, h_avail, nstripes))
		return -EINVAL;
	if (!nkfs_gpu_ready())
		return -EAGAIN;
	if (!nstripes)
		return 0;
	if (!h_parts || !h_blocks || part_pitch < nkfs_part_size(block_size, k) || (part_pitch & 15) ||
	    (nstripes > 1 && block_pitch < block_size))
		return -EINVAL;
	struct hp h = { .dir = HP_DEC, .n = n_slots, .k = k, .n_slots = n_slots, .navail = navail,
			.nstripes = nstripes, .max_block = block_size, .block_size = block_size,
			.block_pitch = nstripes > 1 ? block_pitch : block_size, .part_pitch = part_pitch,
			.blocks = h_blocks, .parts = (uint8_t *)h_parts, .ids = h_ids, .avail = h_avail,
			.expect = h_expect, .badmask = h_expect ? h_badmask : NULL, .status = h_status,
			.chunk = chunk_bytes };
	return hp_run(&h);
}

int nkfs_nk8_decode_ragged_host(const uint8_t *h_parts, const uint64_t *h_part_off, int n_slots,
				const uint8_t *h_ids, const uint8_t *h_avail, int navail, int k, uint8_t *h_blocks,
				const uint64_t *h_block_off, const uint32_t *h_block_size, uint32_t max_block_size,
				uint32_t nstripes, int32_t *h_status, const uint64_t *h_expect, uint64_t *h_badmask,
				uint64_t chunk_bytes)
{
	if (!dec_args_ok(n_slots, navail, k, max_block_size, h_ids, h_avail, nstripes))
		return -EINVAL;
	if (!nkfs_gpu_ready())
		return -EAGAIN;
	if (!nstripes)
		return 0;
	if (!h_parts || !h_part_off || !h_blocks || !h_block_off || !h_block_size ||
	    !ragged_ok(h_block_size, h_block_off, h_part_off, nstripes, max_block_size, n_slots, k))
		return -EINVAL;
	struct hp h = { .dir = HP_DEC, .n = n_slots, .k = k, .n_slots = n_slots, .navail = navail,
			.nstripes = nstripes, .max_block = max_block_size, .sizes = h_block_size,
			.boff = h_block_off, .poff = h_part_off, .blocks = h_blocks, .parts = (uint8_t *)h_parts,
			.ids = h_ids, .avail = h_avail, .expect = h_expect, .badmask = h_expect ? h_badmask : NULL,
			.status = h_status, .chunk = chunk_bytes };
	return hp_run(&h);
}

int nkfs_nk8_decode_pages(const uint8_t *h_parts, const uint64_t *h_part_off, int n_slots, const uint8_t *h_ids,
			  const uint8_t *h_avail, int navail, int k, uint8_t *const *h_pages, uint32_t page_size,
			  const uint64_t *h_first_page, const uint32_t *h_block_size, uint32_t max_block_size,
			  uint32_t nstripes, int32_t *h_status, const uint64_t *h_expect, uint64_t *h_badmask,
			  uint64_t chunk_bytes)
{
	if (!dec_args_ok(n_slots, navail, k, max_block_size, h_ids, h_avail, nstripes))
		return -EINVAL;
	if (!nkfs_gpu_ready())
		return -EAGAIN;
	if (!nstripes)
		return 0;
	if (!h_parts || !h_part_off || !h_block_size || !pages_ok(h_pages, page_size, h_first_page, nstripes) ||
	    !ragged_ok(h_block_size, NULL, h_part_off, nstripes, max_block_size, n_slots, k))
		return -EINVAL;
	struct hp h = { .dir = HP_DEC, .n = n_slots, .k = k, .n_slots = n_slots, .navail = navail,
			.nstripes = nstripes, .max_block = max_block_size, .sizes = h_block_size,
			.poff = h_part_off, .pages = h_pages, .first_page = h_first_page, .page_size = page_size,
			.parts = (uint8_t *)h_parts, .ids = h_ids, .avail = h_avail, .expect = h_expect,
			.badmask = h_expect ? h_badmask : NULL, .status = h_status, .chunk = chunk_bytes };
	return hp_run(&h);
}
