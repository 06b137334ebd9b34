/*
 * pin_probe.c -- what the HIP runtime reports about host memory around the
 * host pipeline's registration lifetime.
 *
 * The pipeline (nkfs_amd/csrc/pipeline.c) trusts the runtime's answer
 * "this range is pinned host memory" (runtime_pinned) and otherwise
 * registers pageable caller memory for the duration of a call.  This probe
 * asks the runtime, with attribute queries only (no DMA into any range whose
 * mapping is in doubt, so it cannot fault), what it reports for:
 *
 *   E1  hipHostMalloc memory (torch pin_memory=True, the trusted case);
 *   E2  a pageable buffer right after a pageable hipMemcpy D2H / H2D (the
 *       runtime may pin pageable memory in place for a large copy and
 *       release that pin later);
 *   E3  the same virtual range after free() + a fresh allocation of the
 *       same size (a recycled address);
 *   E4  two byte-disjoint registrations sharing a 4 KiB page, then the first
 *       unregistered;
 *   E5  a register / unregister / munmap / mmap at the same address;
 *   E6  ROCr's own record (hsa_amd_pointer_info: type, agent base, size,
 *       agents) of the E4 ranges and of the page they share, and of a
 *       pageable buffer after large pageable copies (in-place pins).
 *
 * Build: gcc -O1 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include tools/pin_probe.c \
 *        -L/opt/rocm/lib -lamdhip64 -lhsa-runtime64 -o tools/pin_probe
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#include <hip/hip_runtime_api.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

static const char *mt(int t)
{
	switch (t) {
	case hipMemoryTypeUnregistered: return "unregistered";
	case hipMemoryTypeHost: return "host";
	case hipMemoryTypeDevice: return "device";
	case hipMemoryTypeManaged: return "managed";
	default: return "?";
	}
}

static void show(const char *what, const void *p, size_t bytes)
{
	hipPointerAttribute_t a;
	memset(&a, 0, sizeof(a));
	hipError_t e = hipPointerGetAttributes(&a, p);
	void *base = NULL;
	size_t size = 0;
	hipError_t e2 = hipErrorUnknown;
	if (e == hipSuccess && a.type == hipMemoryTypeHost)
		e2 = hipMemGetAddressRange(&base, &size, a.devicePointer ? a.devicePointer : (void *)p);
	(void)hipGetLastError();
	printf("  %-44s p=%p attr_rc=%d type=%s dev=%p host=%p flags=0x%x", what, p, (int)e,
	       e == hipSuccess ? mt(a.type) : "-", a.devicePointer, a.hostPointer, a.allocationFlags);
	if (e2 == hipSuccess) {
		const uintptr_t dp = (uintptr_t)(a.devicePointer ? a.devicePointer : p);
		printf(" range_base=%p size=%zu off=%zu covers_%zu=%s", base, size, (size_t)(dp - (uintptr_t)base),
		       bytes, dp - (uintptr_t)base + bytes <= size ? "yes" : "NO");
	}
	printf("\n");
}

static const char *pt(int t)
{
	static const char *n[] = { "unknown", "hsa", "locked", "graphics", "ipc", "reserved", "vmem" };
	return t >= 0 && t <= 6 ? n[t] : "?";
}

static void rocr(const char *what, const void *p)
{
	hsa_amd_pointer_info_t in;
	memset(&in, 0, sizeof(in));
	in.size = sizeof(in);
	uint32_t na = 0;
	hsa_agent_t *ag = NULL;
	hsa_status_t s = hsa_amd_pointer_info(p, &in, malloc, &na, &ag);
	printf("  rocr %-39s p=%p rc=%d type=%s agent_base=%p host_base=%p size=%zu agents=%u", what, p, (int)s,
	       pt(in.type), in.agentBaseAddress, in.hostBaseAddress, in.sizeInBytes, na);
	if (in.type != HSA_EXT_POINTER_TYPE_UNKNOWN && in.hostBaseAddress) {
		const uintptr_t hb = (uintptr_t)in.hostBaseAddress;
		printf(" [%#lx, %#lx) contains_p=%s", (unsigned long)hb, (unsigned long)(hb + in.sizeInBytes),
		       (uintptr_t)p >= hb && (uintptr_t)p < hb + in.sizeInBytes ? "yes" : "NO");
	}
	printf("\n");
	free(ag);
}

static hsa_agent_t g_gpu;

static hsa_status_t find_gpu(hsa_agent_t a, void *data)
{
	hsa_device_type_t t;
	(void)data;
	if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_GPU &&
	    !g_gpu.handle)
		g_gpu = a;
	return HSA_STATUS_SUCCESS;
}

/* the GPU's SVM access attribute for the page holding p (KFD's page-granular
 * record; a query only) */
static void svm(const char *what, const void *p)
{
	hsa_amd_svm_attribute_pair_t q[2] = { { HSA_AMD_SVM_ATTRIB_ACCESS_QUERY, g_gpu.handle },
					      { HSA_AMD_SVM_ATTRIB_GLOBAL_FLAG, 0 } };
	void *pg = (void *)((uintptr_t)p & ~4095ul);
	hsa_status_t s = hsa_amd_svm_attributes_get(pg, 4096, q, 2);
	const char *acc = q[0].attribute == HSA_AMD_SVM_ATTRIB_AGENT_ACCESSIBLE ? "accessible"
			  : q[0].attribute == HSA_AMD_SVM_ATTRIB_AGENT_ACCESSIBLE_IN_PLACE ? "in_place"
			  : q[0].attribute == HSA_AMD_SVM_ATTRIB_AGENT_NO_ACCESS ? "NO_ACCESS"
										  : "other";
	printf("  svm  %-39s page=%p rc=%#x gpu_access=%s(%#lx) global_flag=%lu\n", what, pg, (unsigned)s, acc,
	       (unsigned long)q[0].attribute, (unsigned long)q[1].value);
}

int main(void)
{
	if (hipSetDevice(0) != hipSuccess || hsa_init() != HSA_STATUS_SUCCESS) {
		printf("no device\n");
		return 1;
	}
	hsa_iterate_agents(find_gpu, NULL);
	const size_t MB8 = 8u << 20;
	void *d = NULL;
	if (hipMalloc(&d, MB8) != hipSuccess)
		return 1;
	hipMemset(d, 0x5a, MB8);
	hipDeviceSynchronize();

	printf("E1 hipHostMalloc (pinned by its owner)\n");
	void *hm = NULL;
	hipHostMalloc(&hm, MB8, 0);
	show("hipHostMalloc 8 MiB", hm, MB8);
	show("hipHostMalloc +1 MiB", (char *)hm + (1 << 20), 1 << 20);
	svm("hipHostMalloc page", hm);
	rocr("hipHostMalloc", hm);
	hipHostFree(hm);
	show("after hipHostFree", hm, 16);

	for (int dir = 0; dir < 2; dir++) {
		printf("E2 pageable buffer after a pageable %s hipMemcpy (8 MiB, malloc)\n", dir ? "H2D" : "D2H");
		char *pg = malloc(MB8 + 64);
		memset(pg, 1, MB8 + 64);
		char *p = pg + 16; /* page-unaligned, as a numpy/torch CPU buffer may be */
		show("before the copy", p, MB8);
		hipError_t ce = dir ? hipMemcpy(d, p, MB8, hipMemcpyHostToDevice)
				    : hipMemcpy(p, d, MB8, hipMemcpyDeviceToHost);
		printf("  copy rc=%d\n", (int)ce);
		show("after the copy (no sync)", p, MB8);
		show("after the copy, +4 MiB", p + (4u << 20), 1 << 20);
		hipDeviceSynchronize();
		show("after hipDeviceSynchronize", p, MB8);
		/* a stream-ordered copy on a second stream, then its sync */
		hipStream_t st;
		hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
		ce = dir ? hipMemcpyAsync(d, p, MB8, hipMemcpyHostToDevice, st)
			 : hipMemcpyAsync(p, d, MB8, hipMemcpyDeviceToHost, st);
		show("after hipMemcpyAsync, before its sync", p, MB8);
		hipStreamSynchronize(st);
		show("after hipStreamSynchronize", p, MB8);
		hipStreamDestroy(st);
		printf("E3 free() + fresh malloc of the same size\n");
		uintptr_t old = (uintptr_t)pg;
		free(pg);
		char *pg2 = malloc(MB8 + 64);
		printf("  same address: %s\n", (uintptr_t)pg2 == old ? "yes" : "no");
		show("fresh buffer at recycled address", pg2 + 16, MB8);
		hipDeviceSynchronize();
		show("fresh buffer after a device sync", pg2 + 16, MB8);
		free(pg2);
	}

	printf("E4 byte-disjoint registrations sharing a page\n");
	char *m = mmap(NULL, 4 * 4096, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
	memset(m, 0, 4 * 4096);
	char *A = m + 100, *B = m + 4096 + 100;
	size_t nA = 4096 - 50, nB = 2 * 4096 - 110;
	printf("  reg A rc=%d\n", (int)hipHostRegister(A, nA, hipHostRegisterPortable));
	(void)hipGetLastError();
	show("A", A, nA);
	rocr("A", A);
	rocr("shared page (A's 2nd, B's 1st)", m + 4096);
	svm("page 0 (A only)", m);
	svm("page 1 (shared)", m + 4096);
	svm("page 2 (B only, not yet)", m + 8192);
	printf("  reg B rc=%d\n", (int)hipHostRegister(B, nB, hipHostRegisterPortable));
	(void)hipGetLastError();
	show("B", B, nB);
	show("B last byte", B + nB - 1, 1);
	rocr("A", A);
	rocr("B", B);
	rocr("shared page", m + 4096);
	rocr("B's last page", m + 3 * 4096 - 20);
	svm("page 0 (A only)", m);
	svm("page 1 (shared)", m + 4096);
	svm("page 2 (B only)", m + 8192);
	printf("  unreg A rc=%d\n", (int)hipHostUnregister(A));
	(void)hipGetLastError();
	show("A after unreg A", A, nA);
	show("B after unreg A", B, nB);
	rocr("A after unreg A", A);
	rocr("B after unreg A", B);
	rocr("shared page after unreg A", m + 4096);
	rocr("B's last page after unreg A", m + 3 * 4096 - 20);
	svm("page 0 after unreg A", m);
	svm("page 1 (shared, B still registered)", m + 4096);
	svm("page 2 (B only)", m + 8192);
	printf("  unreg B rc=%d\n", (int)hipHostUnregister(B));
	(void)hipGetLastError();
	show("B after unreg B", B, nB);
	svm("page 1 after unreg B", m + 4096);
	svm("page 2 after unreg B", m + 8192);
	printf("E4b nested: register the whole 4 pages, then a range inside at another start\n");
	printf("  reg all rc=%d\n", (int)hipHostRegister(m, 4 * 4096, hipHostRegisterPortable));
	(void)hipGetLastError();
	printf("  reg inner rc=%d\n", (int)hipHostRegister(m + 5000, 3000, hipHostRegisterPortable));
	(void)hipGetLastError();
	show("inner", m + 5000, 3000);
	rocr("inner", m + 5000);
	rocr("outer first page", m);
	svm("outer page 0 (nested)", m);
	svm("outer page 1 (holds inner)", m + 4096);
	printf("  unreg inner rc=%d\n", (int)hipHostUnregister(m + 5000));
	(void)hipGetLastError();
	svm("outer page 0 after unreg inner", m);
	svm("outer page 1 after unreg inner", m + 4096);
	svm("outer page 3 after unreg inner", m + 3 * 4096);
	printf("  unreg all rc=%d\n", (int)hipHostUnregister(m));
	(void)hipGetLastError();
	show("all after both unreg", m, 4 * 4096);

	printf("E5 register / unregister / munmap / mmap at the same address\n");
	printf("  reg rc=%d\n", (int)hipHostRegister(m, 4 * 4096, hipHostRegisterPortable));
	(void)hipGetLastError();
	printf("  unreg rc=%d\n", (int)hipHostUnregister(m));
	(void)hipGetLastError();
	munmap(m, 4 * 4096);
	char *m2 = mmap(m, 4 * 4096, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_FIXED, -1, 0);
	show("remapped range", m2, 4 * 4096);
	munmap(m2, 4 * 4096);

	printf("E6 ROCr record of pageable buffers after large pageable copies\n");
	for (size_t mb = 8; mb <= 64; mb *= 8) {
		const size_t nb = mb << 20;
		void *dd = NULL;
		if (hipMalloc(&dd, nb) != hipSuccess)
			break;
		char *pg = malloc(nb + 64), *p = pg + 16;
		memset(pg, 2, nb + 64);
		printf("  %zu MiB D2H rc=%d\n", mb, (int)hipMemcpy(p, dd, nb, hipMemcpyDeviceToHost));
		rocr("buffer after D2H", p);
		rocr("buffer end after D2H", p + nb - 1);
		svm("buffer first page after D2H", p);
		printf("  %zu MiB H2D rc=%d\n", mb, (int)hipMemcpy(dd, p, nb, hipMemcpyHostToDevice));
		rocr("buffer after H2D", p);
		hipDeviceSynchronize();
		rocr("buffer after device sync", p);
		free(pg);
		hipFree(dd);
	}

	hipFree(d);
	printf("done\n");
	return 0;
}
