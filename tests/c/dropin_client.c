/*
 * dropin_client.c -- a reference-style C caller of libnkfs_crt.so.
 *
 * Uses only the reference's crt/ symbols through include/nkfs_crt.h, the way
 * crt/nk8.c's own self test (crt/nk8.c:601-723) and the client's payload
 * checksum (client/lib/client.c:137-148) use them: nk8_init, random block ->
 * nk8_split_block -> k random distinct parts -> nk8_assemble_block -> csum of
 * input == csum of output; parts released with crt_free.  Exit 0 on success.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "nkfs_crt.h"

static uint64_t csum_of(const void *p, size_t len)
{
	struct csum_ctx ctx;
	struct csum sum;
	csum_reset(&ctx);
	/* feed in uneven pieces like a socket reader would */
	size_t off = 0, step = 1;
	while (off < len) {
		size_t n = len - off < step ? len - off : step;
		csum_update(&ctx, (const char *)p + off, n);
		off += n;
		step = step * 3 + 7;
	}
	csum_digest(&ctx, &sum);
	return csum_u64(&sum);
}

static int round_trip(uint32_t size, int n, int k, unsigned seed)
{
	uint8_t *block = crt_malloc(size), *result = crt_malloc(size);
	uint8_t **parts = NULL, *ids = NULL, *sparts[254], sids[254];
	int err;
	srand(seed);
	for (uint32_t i = 0; i < size; i++)
		block[i] = (uint8_t)rand();
	uint64_t in_sum = csum_of(block, size);
	if (in_sum != XXH64(block, size, 0)) {
		fprintf(stderr, "csum != XXH64\n");
		return 1;
	}
	if ((err = nk8_split_block(block, size, n, k, &parts, &ids))) {
		fprintf(stderr, "split %d\n", err);
		return 1;
	}
	for (int i = 0; i < k; i++) {
		for (;;) {
			int j = rand() % n, used = 0;
			for (int m = 0; m < i; m++)
				used |= sparts[m] == parts[j];
			if (!used) {
				sparts[i] = parts[j];
				sids[i] = ids[j];
				break;
			}
		}
	}
	memset(result, 0, size);
	if ((err = nk8_assemble_block(sparts, sids, k, k, result, size))) {
		fprintf(stderr, "assemble %d\n", err);
		return 1;
	}
	int bad = csum_of(result, size) != in_sum || memcmp(block, result, size);
	for (int i = 0; i < n; i++)
		crt_free(parts[i]);
	crt_free(parts);
	crt_free(ids);
	crt_free(block);
	crt_free(result);
	if (bad)
		fprintf(stderr, "round trip mismatch size %u n %d k %d\n", size, n, k);
	return bad;
}

int main(void)
{
	int err = nk8_init();
	if (err) {
		fprintf(stderr, "nk8_init %d\n", err);
		return 2;
	}
	static const struct { uint32_t size; int n, k; } cases[] = {
		{4096, 4, 2}, {1048576, 8, 5}, {65536, 8, 5}, {70000, 255, 254}, {3000, 16, 12}, {1, 2, 2}, {13, 8, 5},
	};
	int bad = 0;
	for (unsigned i = 0; i < sizeof(cases) / sizeof(cases[0]); i++)
		bad |= round_trip(cases[i].size, cases[i].n, cases[i].k, 1234u + i);
	/* argument errors exactly as crt/nk8.c:356-365 */
	uint8_t **pp;
	uint8_t *pi;
	bad |= nk8_split_block((uint8_t *)"x", 0, 4, 2, &pp, &pi) != -22;
	bad |= nk8_split_block((uint8_t *)"x", 1, 2, 3, &pp, &pi) != -22;
	nk8_release();
	/* still usable after release (its tables stay, as in the reference) */
	bad |= round_trip(5000, 5, 3, 99);
	printf(bad ? "dropin_client: FAIL\n" : "dropin_client: ok\n");
	return bad;
}
