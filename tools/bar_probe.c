/*
 * bar_probe.c -- can the host write device memory directly (the PCIe BAR),
 * and what does a host store / load of it cost?  (a
 * per-call mailbox in device memory, written by the host over the BAR, so
 * only the answer crosses PCIe back.)
 *
 * For hipExtMallocWithFlags(hipDeviceMallocFinegrained) and
 * hipDeviceMallocUncached: the pointer attributes, a host store + load
 * round trip checked through a hipMemcpy D2H, and the mean host cost of a
 * 64-bit store + sfence and of a 64-bit load.  Host-side accesses only; a
 * pointer the host cannot map ends the probe (SIGSEGV in this process), it
 * never touches the GPU's page tables.
 *
 * Build: gcc -O1 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include tools/bar_probe.c \
 *        -L/opt/rocm/lib -lamdhip64 -o tools/bar_probe
 */
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <time.h>

#include <hip/hip_runtime_api.h>


static double now_us(void)
{
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static void try_flag(const char *name, unsigned flags)
{
	void *p = NULL;
	hipError_t e = hipExtMallocWithFlags(&p, 1 << 20, flags);
	printf("%s: alloc rc=%d p=%p\n", name, (int)e, p);
	if (e != hipSuccess) {
		(void)hipGetLastError();
		return;
	}
	hipPointerAttribute_t a;
	memset(&a, 0, sizeof(a));
	e = hipPointerGetAttributes(&a, p);
	printf("  attr rc=%d type=%d dev=%p host=%p flags=0x%x\n", (int)e, (int)a.type, a.devicePointer, a.hostPointer,
	       a.allocationFlags);
	volatile uint64_t *h = (volatile uint64_t *)(a.hostPointer ? a.hostPointer : p);
	fflush(stdout);
	h[0] = 0x1122334455667788ull; /* SIGSEGV here: the host cannot map it */
	__sync_synchronize();
	uint64_t back = 0;
	e = hipMemcpy(&back, p, 8, hipMemcpyDeviceToHost);
	printf("  host store -> device copy: rc=%d value=%#llx (%s)\n", (int)e, (unsigned long long)back,
	       back == 0x1122334455667788ull ? "ok" : "MISMATCH");
	const int N = 20000;
	double t0 = now_us();
	for (int i = 0; i < N; i++) {
		h[i & 63] = (uint64_t)i;
		__builtin_ia32_sfence();
	}
	double t1 = now_us();
	uint64_t acc = 0;
	for (int i = 0; i < N; i++)
		acc += h[(i * 8) & 63];
	double t2 = now_us();
	printf("  host 64-bit store+sfence %.3f us, 64-bit load %.3f us (acc %llu)\n", (t1 - t0) / N, (t2 - t1) / N,
	       (unsigned long long)acc);
	(void)hipFree(p);
}

int main(void)
{
	if (hipSetDevice(0) != hipSuccess) {
		printf("no device\n");
		return 1;
	}
	try_flag("hipDeviceMallocFinegrained", hipDeviceMallocFinegrained);
	try_flag("hipDeviceMallocUncached", hipDeviceMallocUncached);
	printf("done\n");
	return 0;
}
