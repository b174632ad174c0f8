// vramdb.hip — can the host write a burst-server doorbell straight into
// device memory (large BAR), and what does a request round trip cost then?
// (the server's mailbox and request slots live in host
// memory, so the leader's poll and its block read are both dependent PCIe
// reads.)  Not product code: a standalone probe (make -C tools vramdb).
//
// For each allocation kind — hipMalloc, hipExtMallocWithFlags(Finegrained),
// hipExtMallocWithFlags(Uncached) — it reports hipPointerGetAttributes and
// whether a host store / load through the pointer works (a SIGSEGV is caught).
// For each kind the host can write, one resident workgroup then serves
// requests whose doorbell (and a 4 KiB request block) the host writes into
// that device memory, answering through a host-coherent done word, against
// the same protocol with the doorbell and block in host memory (the product's
// layout today, tools/pingpong mode 2).  One JSON line per case.
#include <hip/hip_runtime.h>
#include <setjmp.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define CHECK(x)                                                                          \
	do {                                                                              \
		hipError_t e_ = (x);                                                      \
		if (e_ != hipSuccess) {                                                   \
			fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
			exit(1);                                                          \
		}                                                                         \
	} while (0)

static constexpr int kBlockWords = 512; // 4 KiB request block

struct Door {
	uint64_t seq; // the doorbell: the host writes the request's seq here
	uint64_t pad[15];
};

__device__ __forceinline__ uint64_t sys_ld64(const uint64_t *p)
{
	return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Poll the doorbell; on a new seq read the block (every thread 16 B), sum it,
// answer with the sum and the seq in host memory.
__global__ __launch_bounds__(256) void server(const Door *door, const uint64_t *block, uint64_t *done,
					      uint64_t *answer, uint32_t stop_after)
{
	__shared__ uint64_t seq_s;
	__shared__ uint64_t part[256];
	const int t = threadIdx.x;
	uint64_t last = 0;
	for (uint32_t served = 0; served < stop_after;) {
		if (t == 0) {
			const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
			uint64_t r;
			while ((r = sys_ld64(&door->seq)) == last) {
				if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) { // 200 ms idle
					r = ~0ull;
					break;
				}
				__builtin_amdgcn_s_sleep(1);
			}
			seq_s = r;
			last = r;
		}
		__syncthreads();
		const uint64_t seq = seq_s;
		if (seq == ~0ull)
			break;
		part[t] = sys_ld64(block + 2 * t) + sys_ld64(block + 2 * t + 1);
		__syncthreads();
		if (t == 0) {
			uint64_t s = 0;
			for (int i = 0; i < 256; i++)
				s += part[i];
			__hip_atomic_store(answer, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
			__hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
		}
		served++;
		__syncthreads();
	}
}

static double now()
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static int cmpd(const void *a, const void *b)
{
	double x = *(const double *)a, y = *(const double *)b;
	return x < y ? -1 : x > y;
}

static sigjmp_buf g_jb;
static void on_segv(int) { siglongjmp(g_jb, 1); }

// Can the host store to and load from p?  (SIGSEGV caught)
static bool host_rw(volatile uint64_t *p)
{
	struct sigaction sa, old;
	memset(&sa, 0, sizeof(sa));
	sa.sa_handler = on_segv;
	sigaction(SIGSEGV, &sa, &old);
	bool ok = false;
	if (sigsetjmp(g_jb, 1) == 0) {
		p[0] = 0x1234567890abcdefull;
		ok = p[0] == 0x1234567890abcdefull;
		p[0] = 0;
	}
	sigaction(SIGSEGV, &old, nullptr);
	return ok;
}

// Round trips of one request: block (4 KiB) and doorbell written by the host
// at (door, block), the answer polled in host memory.
static void serve(const char *tag, Door *door, uint64_t *block, double budget, hipStream_t st)
{
	uint64_t *done, *answer, *done_d, *answer_d;
	CHECK(hipHostMalloc((void **)&done, 64, hipHostMallocCoherent));
	CHECK(hipHostMalloc((void **)&answer, 64, hipHostMallocCoherent));
	CHECK(hipHostGetDevicePointer((void **)&done_d, done, 0));
	CHECK(hipHostGetDevicePointer((void **)&answer_d, answer, 0));
	*done = 0;
	door->seq = 0;
	__atomic_thread_fence(__ATOMIC_SEQ_CST);
	const int maxit = 200000;
	double *tm = (double *)malloc(sizeof(double) * maxit), *tw = (double *)malloc(sizeof(double) * maxit);
	uint64_t local[kBlockWords];
	for (int i = 0; i < kBlockWords; i++)
		local[i] = (uint64_t)i * 0x9E3779B97F4A7C15ull;
	hipLaunchKernelGGL(server, dim3(1), dim3(256), 0, st, door, block, done_d, answer_d, (uint32_t)maxit);
	CHECK(hipGetLastError());
	int it = 0, w = 0, bad = 0;
	uint64_t seq = 0;
	const double t0 = now();
	while (it < maxit - 1 && now() - t0 < budget) {
		const double a = now();
		++seq;
		local[0] = seq;
		memcpy(block, local, sizeof(local)); // the request block, rewritten per request
		__atomic_thread_fence(__ATOMIC_SEQ_CST); // block before doorbell (sfence for WC mappings)
		__atomic_store_n(&door->seq, seq, __ATOMIC_RELEASE);
		__atomic_thread_fence(__ATOMIC_SEQ_CST);
		const double b = now();
		bool lost = false;
		while (!lost && __atomic_load_n(done, __ATOMIC_ACQUIRE) != seq)
			lost = now() - a > 0.5;
		if (lost) { // the server never saw the doorbell (or idled out): report, stop
			printf("{\"case\": \"%s\", \"no_answer_to\": %llu}\n", tag, (unsigned long long)seq);
			break;
		}
		uint64_t s = 0;
		for (int i = 0; i < kBlockWords; i++)
			s += local[i];
		bad += __atomic_load_n(answer, __ATOMIC_ACQUIRE) != s;
		if (w++ >= 50) {
			tw[it] = b - a;
			tm[it++] = now() - a;
		}
	}
	door->seq = ~0ull; // the exit word (or the server idles out after 200 ms)
	__atomic_thread_fence(__ATOMIC_SEQ_CST);
	CHECK(hipStreamSynchronize(st));
	if (it == 0) {
		free(tm);
		free(tw);
		return;
	}
	qsort(tm, it, sizeof(double), cmpd);
	qsort(tw, it, sizeof(double), cmpd);
	printf("{\"case\": \"%s\", \"iters\": %d, \"us_median\": %.2f, \"us_p10\": %.2f, \"us_p90\": %.2f, "
	       "\"host_write_us_median\": %.2f, \"bad\": %d}\n",
	       tag, it, tm[it / 2] * 1e6, tm[it / 10] * 1e6, tm[it * 9 / 10] * 1e6, tw[it / 2] * 1e6, bad);
	fflush(stdout);
	free(tm);
	free(tw);
	(void)hipHostFree(done);
	(void)hipHostFree(answer);
}

int main(int argc, char **argv)
{
	const double budget = argc > 1 ? atof(argv[1]) : 0.3;
	hipDeviceProp_t prop;
	CHECK(hipGetDeviceProperties(&prop, 0));
	printf("{\"device\": \"%s\", \"isLargeBar\": %d}\n", prop.gcnArchName, prop.isLargeBar);
	hipStream_t st;
	CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
	const size_t bytes = sizeof(Door) + 8 * kBlockWords;
	// the product's layout: doorbell and block in host-coherent memory (a
	// hipHostMalloc pointer is valid on the device too: unified addresses)
	{
		uint8_t *h;
		CHECK(hipHostMalloc((void **)&h, bytes, hipHostMallocCoherent));
		memset(h, 0, bytes);
		serve("host_coherent", (Door *)h, (uint64_t *)(h + sizeof(Door)), budget, st);
		(void)hipHostFree(h);
	}
	static const struct {
		const char *name;
		unsigned flags; // 0: hipMalloc
	} kinds[3] = {{"hipMalloc", 0}, {"finegrained", hipDeviceMallocFinegrained}, {"uncached", hipDeviceMallocUncached}};
	for (const auto &k : kinds) {
		void *p = nullptr;
		hipError_t e = k.flags ? hipExtMallocWithFlags(&p, bytes, k.flags) : hipMalloc(&p, bytes);
		if (e != hipSuccess) {
			printf("{\"kind\": \"%s\", \"alloc\": \"%s\"}\n", k.name, hipGetErrorString(e));
			continue;
		}
		CHECK(hipMemset(p, 0, bytes));
		CHECK(hipDeviceSynchronize());
		hipPointerAttribute_t at;
		memset(&at, 0, sizeof(at));
		const hipError_t ea = hipPointerGetAttributes(&at, p);
		const bool rw = host_rw((volatile uint64_t *)p);
		printf("{\"kind\": \"%s\", \"attr_rc\": %d, \"type\": %d, \"hostPointer\": \"%p\", \"devicePointer\": \"%p\", "
		       "\"host_rw\": %s}\n",
		       k.name, (int)ea, (int)at.type, at.hostPointer, at.devicePointer, rw ? "true" : "false");
		fflush(stdout);
		if (rw) {
			char tag[64];
			snprintf(tag, sizeof(tag), "vram_%s", k.name);
			serve(tag, (Door *)p, (uint64_t *)((uint8_t *)p + sizeof(Door)), budget, st);
		}
		(void)hipFree(p);
	}
	CHECK(hipStreamDestroy(st));
	return 0;
}
