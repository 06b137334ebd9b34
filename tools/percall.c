/*
 * percall.c -- per-call cost of the drop-in entry points, the calls the
 * reference's unchanged callers make (SURVEY.md §8(b) "Callers"):
 *   csum_reset + csum_update + csum_digest of one buffer
 *       client payload dsum per 64 KiB chunk (client/lib/client.c:146-148),
 *       packet-header sum (crt/net_pkt.c:3-10)
 *   nk8_split_block / nk8_assemble_block of one block (crt/nk8.c:344,446)
 * timed the same way on any library exporting the crt/ symbols: the MI355X
 * library (nkfs_amd/lib/libnkfs_crt.so) and the reference compiled from its
 * own sources (oracle/_ref/libnkfs_ref.so), on the same host core.
 *
 *   gcc -O2 -o tools/percall tools/percall.c -ldl
 *   tools/percall <library.so> [label]
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

struct csum_ctx {
	unsigned char state[88]; /* XXH64_state_t, crt/include/xxhash.h:105 */
};
struct csum {
	uint64_t val;
};

static int (*p_init)(void);
static int (*p_split)(uint8_t *, uint32_t, int, int, uint8_t ***, uint8_t **);
static int (*p_assemble)(uint8_t **, uint8_t *, int, int, uint8_t *, uint32_t);
static void (*p_reset)(struct csum_ctx *);
static void (*p_update)(struct csum_ctx *, const void *, size_t);
static void (*p_digest)(struct csum_ctx *, struct csum *);
static void (*p_free)(void *);

static double now(void)
{
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec + t.tv_nsec * 1e-9;
}

/* median of `reps` timings of `iters` calls, in microseconds per call */
#define TIME_US(iters, reps, ...)                                         \
	({                                                                \
		double best[64];                                          \
		for (int r_ = 0; r_ < (reps); r_++) {                     \
			double t0_ = now();                               \
			for (int i_ = 0; i_ < (iters); i_++) {            \
				__VA_ARGS__;                              \
			}                                                 \
			best[r_] = (now() - t0_) * 1e6 / (iters);          \
		}                                                         \
		for (int a_ = 0; a_ < (reps); a_++)                       \
			for (int b_ = a_ + 1; b_ < (reps); b_++)          \
				if (best[b_] < best[a_]) {                \
					double x_ = best[a_];             \
					best[a_] = best[b_];              \
					best[b_] = x_;                    \
				}                                         \
		best[(reps) / 2];                                         \
	})

int main(int argc, char **argv)
{
	if (argc < 2) {
		fprintf(stderr, "usage: %s <library.so> [label]\n", argv[0]);
		return 2;
	}
	const char *label = argc > 2 ? argv[2] : argv[1];
	void *h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
	if (!h) {
		fprintf(stderr, "%s\n", dlerror());
		return 1;
	}
	void (*loglvl)(int) = (void (*)(int))dlsym(h, "crt_log_set_level");
	if (loglvl)
		loglvl(10); /* reference: keep its log file out of the timings */
	p_init = (int (*)(void))dlsym(h, "nk8_init");
	p_split = (int (*)(uint8_t *, uint32_t, int, int, uint8_t ***, uint8_t **))dlsym(h, "nk8_split_block");
	p_assemble = (int (*)(uint8_t **, uint8_t *, int, int, uint8_t *, uint32_t))dlsym(h, "nk8_assemble_block");
	p_reset = (void (*)(struct csum_ctx *))dlsym(h, "csum_reset");
	p_update = (void (*)(struct csum_ctx *, const void *, size_t))dlsym(h, "csum_update");
	p_digest = (void (*)(struct csum_ctx *, struct csum *))dlsym(h, "csum_digest");
	p_free = (void (*)(void *))dlsym(h, "crt_free");
	if (!p_init || !p_split || !p_assemble || !p_reset || !p_update || !p_digest || !p_free) {
		fprintf(stderr, "missing symbols in %s\n", argv[1]);
		return 1;
	}
	if (p_init()) {
		fprintf(stderr, "nk8_init failed\n");
		return 1;
	}
	/* PERCALL_SVC=1 / 2: the product's opt-in resident service wave for
	 * the per-call digests, mailbox in host memory / in device memory
	 * written over the BAR (nkfs_percall_service; absent in the reference) */
	if (getenv("PERCALL_SVC")) {
		int (*svc)(int) = (int (*)(int))dlsym(h, "nkfs_percall_service");
		if (!svc || svc(atoi(getenv("PERCALL_SVC")))) {
			fprintf(stderr, "nkfs_percall_service unavailable\n");
			return 1;
		}
	}
	const size_t maxb = 1u << 20;
	uint8_t *buf = malloc(maxb), *out = malloc(maxb);
	for (size_t i = 0; i < maxb; i++)
		buf[i] = (uint8_t)(i * 2654435761u >> 13);
	uint64_t sink = 0;

	static const size_t csz[] = {64, 1024, 65536, 1048576};
	for (unsigned c = 0; c < sizeof(csz) / sizeof(csz[0]); c++) {
		const size_t len = csz[c];
		const int iters = len >= 1048576 ? 20 : 200;
		double us = TIME_US(iters, 7, {
			struct csum_ctx ctx;
			struct csum s;
			p_reset(&ctx);
			p_update(&ctx, buf, len);
			p_digest(&ctx, &s);
			sink ^= s.val;
		});
		printf("%-10s csum %8zu B          %10.2f us/call  %8.3f GB/s\n", label, len, us, len / us / 1e3);
	}

	static const struct { uint32_t B; int n, k; } ec[] = {
		{4096, 4, 2}, {65536, 8, 5}, {1048576, 8, 5},
	};
	for (unsigned c = 0; c < sizeof(ec) / sizeof(ec[0]); c++) {
		const uint32_t B = ec[c].B;
		const int n = ec[c].n, k = ec[c].k;
		const int iters = B >= 1048576 ? 10 : 100;
		double us = TIME_US(iters, 5, {
			uint8_t **parts, *ids;
			if (p_split(buf, B, n, k, &parts, &ids)) {
				fprintf(stderr, "split failed\n");
				exit(1);
			}
			for (int i = 0; i < n; i++)
				p_free(parts[i]);
			p_free(parts);
			p_free(ids);
		});
		printf("%-10s split    %8u B N%dK%d  %10.2f us/call  %8.3f GB/s\n", label, B, n, k, us, B / us / 1e3);
		uint8_t **parts, *ids;
		if (p_split(buf, B, n, k, &parts, &ids))
			return 1;
		uint8_t *sp[8], sid[8];
		for (int i = 0; i < k; i++) { /* the last k parts: every one a real decode */
			sp[i] = parts[n - 1 - i];
			sid[i] = ids[n - 1 - i];
		}
		us = TIME_US(iters, 5, {
			if (p_assemble(sp, sid, k, k, out, B)) {
				fprintf(stderr, "assemble failed\n");
				exit(1);
			}
		});
		if (memcmp(out, buf, B)) {
			fprintf(stderr, "assemble mismatch\n");
			return 1;
		}
		printf("%-10s assemble %8u B N%dK%d  %10.2f us/call  %8.3f GB/s\n", label, B, n, k, us, B / us / 1e3);
		for (int i = 0; i < n; i++)
			p_free(parts[i]);
		p_free(parts);
		p_free(ids);
	}
	fprintf(stderr, "sink %llx\n", (unsigned long long)sink);
	return 0;
}
