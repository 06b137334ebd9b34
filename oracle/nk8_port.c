/*
 * oracle/nk8_port.c -- CPU restatement of the nkfs N-K erasure code and
 * XXH64 checksum, used ONLY as test infrastructure (the parity checker and
 * the bench's cpu_baseline "port" leg).  Nothing in nkfs_amd/ links, loads or
 * calls this file; the product path is the HIP library under nkfs_amd/csrc.
 *
 * Pinned by: tests/golden/ fixtures generated from the reference's own
 * crt/nk8.c + crt/xxhash.c compiled by oracle/ref/Makefile, and by the
 * independent python `xxhash` module (tests/test_oracle.py).
 *
 * Reference algorithm followed (file:line under irqlevel/nkfs crt/):
 *   GF(2^8) multiply, reduction poly 0x11B ........ nk8.c:54-74
 *   product table gf_log[a][b] = a*b .............. nk8.c:4-8, 94-109
 *   division table gf_alog[a][b] = a/b ............ nk8.c:76-92, 111-122
 *   part size / tail handling ..................... nk8.c:311-317, 393-398
 *   id rule (distinct, 1..255, rejection) ......... nk8.c:319-342, random.c:15-33
 *   encode (Vandermonde row ids[i]^m) ............. nk8.c:403-421
 *   decode (first k distinct ids, V^-1, apply) .... nk8.c:509-582
 *   Gauss-Jordan inverse .......................... nk8.c:199-266
 *   XXH64 one-shot / streaming .................... xxhash.c:358-496, 566-577,
 *                                                   736-836, 838-930
 * The restatement keeps the reference's loop order (n passes over the block,
 * one product-table lookup per term) so that its timing is a faithful CPU
 * baseline, but takes the part ids as an explicit argument so that outputs
 * are reproducible.
 */
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <fcntl.h>
#include <unistd.h>

typedef uint8_t u8;
typedef uint32_t u32;
typedef uint64_t u64;

#define ORC_MIN_K 2
#define ORC_MAX_K 254
#define ORC_MIN_N 2
#define ORC_MAX_N 255

static u8 orc_mul[256][256]; /* orc_mul[a][b] = a*b in GF(2^8)/0x11B */
static u8 orc_div[256][256]; /* orc_div[a][b] = a/b, 0 when a or b is 0 */
static int orc_ready;

/* Carry-less product of two bytes followed by reduction modulo
 * x^8+x^4+x^3+x+1.  Same field and polynomial as nk8.c:54-74. */
static u8 orc_gf_mul_slow(u8 a, u8 b)
{
	u32 acc = 0;
	for (int bit = 0; bit < 8; bit++)
		if (b & (1u << bit))
			acc ^= (u32)a << bit;
	for (int bit = 14; bit >= 8; bit--)
		if (acc & (1u << bit))
			acc ^= 0x11Bu << (bit - 8);
	return (u8)acc;
}

int orc_init(void)
{
	if (orc_ready)
		return 0;
	for (int a = 0; a < 256; a++)
		for (int b = 0; b < 256; b++)
			orc_mul[a][b] = orc_gf_mul_slow((u8)a, (u8)b);
	/* a/b = the unique q with q*b == a (nk8.c:76-92 finds it by search) */
	memset(orc_div, 0, sizeof(orc_div));
	for (int q = 1; q < 256; q++)
		for (int b = 1; b < 256; b++)
			orc_div[orc_mul[q][b]][b] = (u8)q;
	orc_ready = 1;
	return 0;
}

u8 orc_gf_mul(u8 a, u8 b) { return orc_mul[a][b]; }
u8 orc_gf_div(u8 a, u8 b) { return orc_div[a][b]; }
const u8 *orc_mul_table(void) { return &orc_mul[0][0]; }

u32 orc_part_size(u32 block_size, int k)
{
	return block_size / (u32)k + ((block_size % (u32)k) ? 1u : 0u);
}

static int orc_bad_params(u32 block_size, int n, int k)
{
	return n < ORC_MIN_N || k < ORC_MIN_K || block_size == 0 || n < k ||
	       n > ORC_MAX_N || k > ORC_MAX_K;
}

/*
 * Encode one block into n planar parts of part_size bytes each, part i at
 * parts + i*part_pitch.  ids[i] is the evaluation point of part i.
 * part_i[j] = XOR_m ids[i]^m * d[j*k+m], d = block zero-padded to ps*k.
 */
int orc_encode(const u8 *block, u32 block_size, int n, int k, const u8 *ids,
	       u8 *parts, u64 part_pitch)
{
	if (orc_bad_params(block_size, n, k))
		return -EINVAL;
	if (!orc_ready)
		return -EAGAIN;
	u32 ps = orc_part_size(block_size, k);
	u32 full_rows = ps;
	u32 tail_len = 0;
	u8 tail[ORC_MAX_K];
	if ((u64)ps * (u32)k > block_size) {
		full_rows = ps - 1;
		tail_len = block_size - full_rows * (u32)k;
		memset(tail, 0, sizeof(tail));
		memcpy(tail, block + (u64)full_rows * k, tail_len);
	}
	u8 row_coef[ORC_MAX_K];
	for (int i = 0; i < n; i++) {
		u8 *out = parts + (u64)i * part_pitch;
		row_coef[0] = 1;
		for (int m = 1; m < k; m++)
			row_coef[m] = orc_mul[row_coef[m - 1]][ids[i]];
		const u8 *src = block;
		for (u32 j = 0; j < full_rows; j++, src += k) {
			u8 acc = 0;
			for (int m = 0; m < k; m++)
				acc ^= orc_mul[row_coef[m]][src[m]];
			out[j] = acc;
		}
		if (tail_len) {
			u8 acc = 0;
			for (int m = 0; m < k; m++)
				acc ^= orc_mul[row_coef[m]][tail[m]];
			out[full_rows] = acc;
		}
	}
	return 0;
}

/* In-place k x k inverse by Gauss-Jordan with row pivoting (nk8.c:199-266
 * pivots nothing -- its gf_swap is a no-op -- which is harmless for the
 * Vandermonde matrices decode builds; a true pivot gives the same unique
 * inverse).  a and inv are row-major k*k.  Returns -EFAULT if singular. */
int orc_invert(u8 *a, u8 *inv, int k)
{
	for (int r = 0; r < k; r++)
		for (int c = 0; c < k; c++)
			inv[r * k + c] = (r == c);
	for (int col = 0; col < k; col++) {
		int piv = -1;
		for (int r = col; r < k; r++)
			if (a[r * k + col]) { piv = r; break; }
		if (piv < 0)
			return -EFAULT;
		if (piv != col) {
			for (int c = 0; c < k; c++) {
				u8 t = a[piv * k + c]; a[piv * k + c] = a[col * k + c]; a[col * k + c] = t;
				t = inv[piv * k + c]; inv[piv * k + c] = inv[col * k + c]; inv[col * k + c] = t;
			}
		}
		u8 p = a[col * k + col];
		for (int c = 0; c < k; c++) {
			a[col * k + c] = orc_div[a[col * k + c]][p];
			inv[col * k + c] = orc_div[inv[col * k + c]][p];
		}
		for (int r = 0; r < k; r++) {
			if (r == col || !a[r * k + col])
				continue;
			u8 f = a[r * k + col];
			for (int c = 0; c < k; c++) {
				a[r * k + c] ^= orc_mul[f][a[col * k + c]];
				inv[r * k + c] ^= orc_mul[f][inv[col * k + c]];
			}
		}
	}
	return 0;
}

/*
 * Decode: parts[c] / ids[c] for c < navail in caller order.  The first k
 * parts with distinct ids are used (nk8.c:509-530); fewer than k distinct
 * -> -EINVAL.  Writes exactly block_size bytes.
 */
int orc_decode(const u8 *const *parts, const u8 *ids, int navail, int k,
	       u8 *block, u32 block_size)
{
	if (orc_bad_params(block_size, navail, k))
		return -EINVAL;
	if (!orc_ready)
		return -EAGAIN;
	const u8 *use[ORC_MAX_K];
	u8 x[ORC_MAX_K];
	int have = 0;
	for (int c = 0; c < navail && have < k; c++) {
		int dup = 0;
		for (int d = 0; d < c; d++)
			if (ids[d] == ids[c]) { dup = 1; break; }
		if (dup)
			continue;
		x[have] = ids[c];
		use[have] = parts[c];
		have++;
	}
	if (have < k)
		return -EINVAL;
	u8 *v = malloc((size_t)k * k), *w = malloc((size_t)k * k);
	if (!v || !w) { free(v); free(w); return -ENOMEM; }
	/* V[m][c] = x_c^m (nk8.c:509-544) */
	for (int c = 0; c < k; c++) {
		u8 p = 1;
		for (int m = 0; m < k; m++) {
			v[m * k + c] = p;
			p = orc_mul[p][x[c]];
		}
	}
	int err = orc_invert(v, w, k);
	if (err) { free(v); free(w); return err; }
	u32 ps = orc_part_size(block_size, k);
	for (u32 j = 0; j < ps; j++) {
		for (int m = 0; m < k; m++) {
			u64 pos = (u64)j * k + m;
			if (pos >= block_size)
				break;
			u8 acc = 0;
			for (int c = 0; c < k; c++)
				acc ^= orc_mul[use[c][j]][w[c * k + m]];
			block[pos] = acc;
		}
	}
	free(v);
	free(w);
	return 0;
}

/* ---------------------------------------------------------------- XXH64 */

#define XP1 0x9E3779B185EBCA87ULL
#define XP2 0xC2B2AE3D27D4EB4FULL
#define XP3 0x165667B19E3779F9ULL
#define XP4 0x85EBCA77C2B2AE63ULL
#define XP5 0x27D4EB2F165667C5ULL

static inline u64 rotl64(u64 v, int r) { return (v << r) | (v >> (64 - r)); }
static inline u64 ld64(const u8 *p) { u64 v; memcpy(&v, p, 8); return v; }
static inline u32 ld32(const u8 *p) { u32 v; memcpy(&v, p, 4); return v; }
static inline u64 xround(u64 acc, u64 w) { return rotl64(acc + w * XP2, 31) * XP1; }
static inline u64 xmerge(u64 h, u64 v) { return (h ^ xround(0, v)) * XP1 + XP4; }

static u64 xfinish(u64 h, const u8 *p, size_t left)
{
	while (left >= 8) {
		h = rotl64(h ^ xround(0, ld64(p)), 27) * XP1 + XP4;
		p += 8; left -= 8;
	}
	if (left >= 4) {
		h = rotl64(h ^ ((u64)ld32(p) * XP1), 23) * XP2 + XP3;
		p += 4; left -= 4;
	}
	while (left--) {
		h = rotl64(h ^ ((u64)(*p++) * XP5), 11) * XP1;
	}
	h ^= h >> 33; h *= XP2;
	h ^= h >> 29; h *= XP3;
	h ^= h >> 32;
	return h;
}

u64 orc_xxh64(const void *input, size_t len, u64 seed)
{
	const u8 *p = input;
	u64 h;
	size_t left = len;
	if (len >= 32) {
		u64 a = seed + XP1 + XP2, b = seed + XP2, c = seed, d = seed - XP1;
		while (left >= 32) {
			a = xround(a, ld64(p));
			b = xround(b, ld64(p + 8));
			c = xround(c, ld64(p + 16));
			d = xround(d, ld64(p + 24));
			p += 32; left -= 32;
		}
		h = rotl64(a, 1) + rotl64(b, 7) + rotl64(c, 12) + rotl64(d, 18);
		h = xmerge(h, a); h = xmerge(h, b); h = xmerge(h, c); h = xmerge(h, d);
	} else {
		h = seed + XP5;
	}
	h += (u64)len;
	return xfinish(h, p, left);
}

/* ------------------------------------------------------ CPU-baseline leg */

/* The reference's split entry point, restated with its allocation pattern
 * (crt_malloc per part, caller frees) and id rule (random distinct 1..255
 * drawn by rejection from /dev/urandom, one open() per draw as in
 * crt/user/crt.c:175-186).  Used only to time the reference's behaviour on
 * the GPU box's host cores. */
static int orc_urandom_u64(u64 *out)
{
	int fd = open("/dev/urandom", O_RDONLY);
	if (fd < 0)
		return -errno;
	ssize_t r = read(fd, out, sizeof(*out));
	close(fd);
	return r == (ssize_t)sizeof(*out) ? 0 : -EIO;
}

int orc_split_block(const u8 *block, u32 block_size, int n, int k,
		    u8 ***pparts, u8 **pids)
{
	if (orc_bad_params(block_size, n, k))
		return -EINVAL;
	if (!orc_ready)
		return -EAGAIN;
	u32 ps = orc_part_size(block_size, k);
	u8 *ids = malloc((size_t)n);
	u8 **parts = calloc((size_t)n, sizeof(u8 *));
	if (!ids || !parts)
		goto nomem;
	for (int i = 0; i < n; i++)
		if (!(parts[i] = malloc(ps)))
			goto nomem;
	for (int i = 0; i < n; i++) {
		for (;;) {
			u64 r;
			if (orc_urandom_u64(&r))
				goto nomem;
			u32 v = (u32)(r & 0xFF);
			if (v >= 255)
				continue;
			u8 cand = (u8)(1 + v);
			int dup = 0;
			for (int j = 0; j < i; j++)
				dup |= ids[j] == cand;
			if (!dup) { ids[i] = cand; break; }
		}
	}
	u8 *row_coef = malloc(ORC_MAX_K);
	if (!row_coef)
		goto nomem;
	/* planar encode straight into the per-part buffers */
	u32 full_rows = ((u64)ps * k > block_size) ? ps - 1 : ps;
	u32 tail_len = block_size - full_rows * (u32)k;
	u8 tail[ORC_MAX_K] = {0};
	memcpy(tail, block + (u64)full_rows * k, tail_len);
	for (int i = 0; i < n; i++) {
		row_coef[0] = 1;
		for (int m = 1; m < k; m++)
			row_coef[m] = orc_mul[row_coef[m - 1]][ids[i]];
		const u8 *src = block;
		u8 *out = parts[i];
		for (u32 j = 0; j < full_rows; j++, src += k) {
			u8 acc = 0;
			for (int m = 0; m < k; m++)
				acc ^= orc_mul[row_coef[m]][src[m]];
			out[j] = acc;
		}
		if (tail_len) {
			u8 acc = 0;
			for (int m = 0; m < k; m++)
				acc ^= orc_mul[row_coef[m]][tail[m]];
			out[full_rows] = acc;
		}
	}
	free(row_coef);
	*pparts = parts;
	*pids = ids;
	return 0;
nomem:
	if (parts)
		for (int i = 0; i < n; i++)
			free(parts[i]);
	free(parts);
	free(ids);
	return -ENOMEM;
}

void orc_free(void *p) { free(p); }

/*
 * Bench harness: encode + XXH64 of every part for `count` blocks of
 * block_size bytes laid out back to back in `blocks`, over `threads`
 * pthreads (stripes are independent).  `split` and `hash` are the entry
 * points timed -- either this file's restatement or the compiled reference
 * (oracle/_ref), passed in as function pointers by the caller.
 * Returns seconds of wall time, or a negative errno.
 */
typedef int (*orc_split_fn)(const u8 *, u32, int, int, u8 ***, u8 **);
typedef u64 (*orc_hash_fn)(const void *, size_t, u64);
typedef void (*orc_free_fn)(void *);
typedef int (*orc_assemble_fn)(u8 **, u8 *, int, int, u8 *, u32);

struct orc_job {
	orc_assemble_fn assemble;
	const u8 *survivors; /* [count][k] part slots to decode from, or NULL */
	u8 *scratch;
	orc_split_fn split;
	orc_hash_fn hash;
	orc_free_fn release;
	const u8 *blocks;
	u32 block_size;
	int n, k;
	u64 first, last;
	u64 digest_xor;
	int err;
};

static void *orc_worker(void *arg)
{
	struct orc_job *job = arg;
	u32 ps = orc_part_size(job->block_size, job->k);
	for (u64 s = job->first; s < job->last; s++) {
		u8 **parts = NULL, *ids = NULL;
		int err = job->split(job->blocks + s * job->block_size,
				     job->block_size, job->n, job->k, &parts, &ids);
		if (err) { job->err = err; return NULL; }
		for (int i = 0; i < job->n; i++)
			job->digest_xor ^= job->hash(parts[i], ps, 0);
		if (job->assemble) {
			u8 *sp[ORC_MAX_K], sid[ORC_MAX_K];
			const u8 *sv = job->survivors + s * (u64)job->k;
			for (int c = 0; c < job->k; c++) {
				sp[c] = parts[sv[c]];
				sid[c] = ids[sv[c]];
			}
			err = job->assemble(sp, sid, job->k, job->k, job->scratch, job->block_size);
			if (err) { job->err = err; return NULL; }
			job->digest_xor ^= job->scratch[job->block_size - 1];
		}
		for (int i = 0; i < job->n; i++)
			job->release(parts[i]);
		job->release(parts);
		job->release(ids);
	}
	return NULL;
}

#include <time.h>
/* The restatement's nk8_assemble_block-shaped entry point. */
int orc_assemble_block(u8 **parts, u8 *ids, int n, int k, u8 *block, u32 block_size)
{
	return orc_decode((const u8 *const *)parts, ids, n, k, block, block_size);
}

/* encode + XXH64 of every part and, when `assemble` is given, decode of
 * every stripe from survivors[s][0..k) (the metric's encode+decode) */
double orc_bench_encode_decode(orc_split_fn split, orc_hash_fn hash,
			       orc_free_fn release, orc_assemble_fn assemble,
			       const u8 *survivors, const u8 *blocks,
			       u32 block_size, int n, int k, u64 count,
			       int threads, u64 *digest_xor)
{
	if (threads < 1)
		threads = 1;
	if (threads > 256)
		threads = 256;
	struct orc_job jobs[256];
	pthread_t tid[256];
	struct timespec t0, t1;
	clock_gettime(CLOCK_MONOTONIC, &t0);
	for (int t = 0; t < threads; t++) {
		jobs[t] = (struct orc_job){ assemble, survivors,
			assemble ? malloc(block_size) : NULL, split, hash,
			release, blocks, block_size, n, k, count * t / threads,
			count * (t + 1) / threads, 0, 0 };
		pthread_create(&tid[t], NULL, orc_worker, &jobs[t]);
	}
	u64 dx = 0;
	int err = 0;
	for (int t = 0; t < threads; t++) {
		pthread_join(tid[t], NULL);
		free(jobs[t].scratch);
		dx ^= jobs[t].digest_xor;
		if (jobs[t].err)
			err = jobs[t].err;
	}
	clock_gettime(CLOCK_MONOTONIC, &t1);
	if (digest_xor)
		*digest_xor = dx;
	if (err)
		return (double)err;
	return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
