/* runtime.h -- host-side context shared by runtime.c, nk8.c and csum.c. */
#ifndef NKFS_RUNTIME_H
#define NKFS_RUNTIME_H

#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime_api.h>

#define NKFS_MAX_DEVICES 16

struct nkfs_ctx {
	int dev;      /* device the stream and scratch belong to */
	hipStream_t stream;
	void *dbuf;   /* device scratch */
	size_t dcap;
	void *hbuf;   /* pinned host scratch */
	size_t hcap;
	hipEvent_t ev[2]; /* created on first use (nkfs_ctx_events) */
	int nev;
	uint64_t seq;     /* completion words handed out on this context */
	volatile uint64_t *done; /* pinned completion word (nkfs_ctx_wait; first use) */
	void *ddone;      /* its device-visible address */
	struct nkfs_ctx *next;
};

struct nkfs_ctx *nkfs_ctx_get(void);          /* on the library's device */
struct nkfs_ctx *nkfs_ctx_get_on(int dev);
void nkfs_ctx_put(struct nkfs_ctx *c);
int nkfs_ctx_dev(struct nkfs_ctx *c, size_t bytes, void **out);
int nkfs_ctx_host(struct nkfs_ctx *c, size_t bytes, void **out);
int nkfs_ctx_events(struct nkfs_ctx *c); /* c->ev[0..1] exist afterwards */
/* everything enqueued on c->stream is done: a spin on a stream-written word
 * when `spin`, else the stream sync (runtime.c) */
int nkfs_ctx_wait(struct nkfs_ctx *c, int spin);
const void *nkfs_gf(void);                   /* tables on the library's device */
const void *nkfs_gf_on(int dev);
const void *nkfs_gf_for(void *stream);       /* tables on the device of `stream` */
int nkfs_use_device(int dev);
void nkfs_gpu_release(void);
void nkfs_ctx_trim(void);
int nkfs_bad_params(uint32_t block_size, int n, int k);
int nkfs_hip_fail(const char *what, int err);
uint64_t nkfs_ctx_outstanding(void); /* contexts taken and not yet put back */
int nkfs_host_depth(void); /* struct nkfs_tune.host_depth: sub-batches in flight per lane */
int nkfs_host_lanes(void); /* struct nkfs_tune.host_lanes: host lanes per device */

#endif
