// pingpong.hip — what a host <-> GPU request round trip costs on this box,
// to size the burst server's request protocol (cgck_group.hip).  Not product
// code: a standalone program (hipcc) run by tools/gpu_*.sh.
//
// One resident workgroup polls a host-coherent mailbox; per mode it answers
// a request after:
//   0  nothing (poll + answer: the bare handshake)
//   1  a system-scope acquire and release fence (the server's fences today)
//   2  one wide read of a 4 KiB request block (every thread 16 B)
//   3  2 + 64 eight-byte answers, agent-scope release, then seq_done
//   4  2 + 64 tagged eight-byte answers, no seq_done (the host checks tags)
//   5  three dependent reads (header -> descriptor -> packet bytes), as the
//      server's request walk does today, then seq_done
//   6  3 with a system-scope release instead of agent scope
// and, for comparison, a launch + hipStreamSynchronize of an empty kernel and
// of a kernel reading the same 4 KiB block.  Prints one JSON line per mode.
#include <hip/hip_runtime.h>
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

struct Box {
	uint32_t seq_req;
	uint32_t pad0[15];
	uint32_t seq_done;
	uint32_t pad1[15];
	uint32_t stop;
	uint32_t mode;
	uint32_t pad2[14];
};

static constexpr int kReqWords = 512; // u64 words: 4 KiB request block
static constexpr int kResp = 64;

__device__ __forceinline__ uint32_t sys_ld32(const uint32_t *p)
{
	return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t raw_ld64(const uint64_t *p)
{
	return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void raw_st64(uint64_t *p, uint64_t v)
{
	__hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void server(Box *box, const uint64_t *req, uint64_t *resp)
{
	__shared__ uint32_t cmd, seq_s;
	__shared__ uint64_t part[256];
	uint32_t last = 0;
	const int t = threadIdx.x;
	const uint32_t mode = box->mode;
	for (;;) {
		if (t == 0) {
			const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
			uint32_t c = 0;
			while (c == 0) {
				const uint32_t r = sys_ld32(&box->seq_req);
				if (sys_ld32(&box->stop))
					c = 2;
				else if (r != last)
					c = 1, last = r;
				else if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) // 200 ms idle
					c = 2;
			}
			cmd = c;
			seq_s = last;
		}
		__syncthreads();
		if (cmd == 2)
			break;
		const uint32_t seq = seq_s;
		uint64_t acc = 0;
		if (mode == 1)
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
		if (mode >= 2 && mode != 5) {
			acc = raw_ld64(req + 2 * t) + raw_ld64(req + 2 * t + 1);
		} else if (mode == 5) {
			const uint64_t h = raw_ld64(req);                     // header
			const uint64_t d = raw_ld64(req + 1 + (h & 7));        // descriptor
			acc = raw_ld64(req + 16 + ((d + t) & 255));            // packet bytes
		}
		if (mode >= 2) {
			part[t] = acc;
			__syncthreads();
			if (t < kResp) {
				uint64_t s = part[t] + part[t + 64] + part[t + 128] + part[t + 192];
				if (mode == 4)
					raw_st64(resp + t, (s & 0xffffffffffull) | ((uint64_t)(seq & 0xffffffu) << 40));
				else if (mode == 3 || mode == 6)
					raw_st64(resp + t, s);
			}
		}
		if (mode == 3)
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
		if (mode == 1 || mode == 6)
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
		__syncthreads();
		if (t == 0 && mode != 4)
			__hip_atomic_store(&box->seq_done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
	}
}

__global__ void empty_kernel() {}

__global__ __launch_bounds__(256) void read_kernel(const uint64_t *req, uint64_t *out)
{
	const uint64_t v = raw_ld64(req + 2 * threadIdx.x) + raw_ld64(req + 2 * threadIdx.x + 1);
	if (v == 0x123456789ull)
		out[threadIdx.x] = v;
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

int main(int argc, char **argv)
{
	const double budget = argc > 1 ? atof(argv[1]) : 0.3;
	const int maxit = 200000;
	double *tm = (double *)malloc(sizeof(double) * maxit);
	Box *box;
	uint64_t *req, *resp;
	CHECK(hipHostMalloc((void **)&box, sizeof(Box), hipHostMallocCoherent));
	CHECK(hipHostMalloc((void **)&req, 8 * kReqWords, hipHostMallocCoherent));
	CHECK(hipHostMalloc((void **)&resp, 8 * kResp, hipHostMallocCoherent));
	Box *box_d;
	uint64_t *req_d, *resp_d, *dout;
	CHECK(hipHostGetDevicePointer((void **)&box_d, box, 0));
	CHECK(hipHostGetDevicePointer((void **)&req_d, req, 0));
	CHECK(hipHostGetDevicePointer((void **)&resp_d, resp, 0));
	CHECK(hipMalloc((void **)&dout, 8 * 256));
	hipStream_t st;
	CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
	uint64_t local[kReqWords];
	for (int i = 0; i < kReqWords; i++)
		local[i] = (uint64_t)i * 0x9E3779B97F4A7C15ull;
	for (uint32_t mode = 0; mode <= 6; mode++) {
		memset(box, 0, sizeof(Box));
		memset(resp, 0, 8 * kResp);
		box->mode = mode;
		hipLaunchKernelGGL(server, dim3(1), dim3(256), 0, st, box_d, req_d, resp_d);
		CHECK(hipGetLastError());
		int it = 0, w = 0, bad = 0;
		uint32_t seq = 0;
		const double t0 = now();
		while (it < maxit && now() - t0 < budget) {
			const double a = now();
			++seq;
			if (mode >= 2) {
				local[0] = seq;
				memcpy(req, local, sizeof(local)); // the request block, rewritten per request
			}
			if (mode == 4)
				for (int i = 0; i < kResp; i++)
					__atomic_store_n(&resp[i], 0ull, __ATOMIC_RELAXED);
			__atomic_store_n(&box->seq_req, seq, __ATOMIC_RELEASE);
			const double give_up = a + 1.0;
			if (mode == 4) {
				for (int i = 0; i < kResp; i++)
					while ((__atomic_load_n(&resp[i], __ATOMIC_ACQUIRE) >> 40) != (seq & 0xffffffu))
						if (now() > give_up) {
							fprintf(stderr, "mode %u: no answer to %u\n", mode, seq);
							return 1;
						}
			} else {
				while (__atomic_load_n(&box->seq_done, __ATOMIC_ACQUIRE) != seq)
					if (now() > give_up) {
						fprintf(stderr, "mode %u: no answer to %u\n", mode, seq);
						return 1;
					}
			}
			if (mode == 3 || mode == 6) {
				// answer i = sum of request words 2i, 2i+1 over the 4 threads i, i+64, ...
				uint64_t s = 0;
				for (int k = 0; k < 4; k++)
					s += local[2 * (0 + 64 * k)] + local[2 * (0 + 64 * k) + 1];
				bad += resp[0] != s;
			}
			if (w++ >= 50)
				tm[it++] = now() - a;
		}
		__atomic_store_n(&box->stop, 1u, __ATOMIC_RELEASE);
		CHECK(hipStreamSynchronize(st));
		qsort(tm, it, sizeof(double), cmpd);
		printf("{\"mode\": %u, \"iters\": %d, \"us_median\": %.2f, \"us_p10\": %.2f, \"us_p90\": %.2f, \"bad\": %d}\n",
		       mode, it, tm[it / 2] * 1e6, tm[it / 10] * 1e6, tm[it * 9 / 10] * 1e6, bad);
		fflush(stdout);
	}
	for (int k = 0; k < 2; k++) {
		int it = 0, w = 0;
		const double t0 = now();
		while (it < maxit && now() - t0 < budget) {
			const double a = now();
			if (k == 0)
				hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st);
			else
				hipLaunchKernelGGL(read_kernel, dim3(1), dim3(256), 0, st, req_d, dout);
			CHECK(hipStreamSynchronize(st));
			if (w++ >= 50)
				tm[it++] = now() - a;
		}
		qsort(tm, it, sizeof(double), cmpd);
		printf("{\"mode\": \"%s\", \"iters\": %d, \"us_median\": %.2f, \"us_p10\": %.2f, \"us_p90\": %.2f}\n",
		       k ? "launch_read4k_sync" : "launch_empty_sync", it, tm[it / 2] * 1e6, tm[it / 10] * 1e6,
		       tm[it * 9 / 10] * 1e6);
		fflush(stdout);
	}
	CHECK(hipStreamDestroy(st));
	return 0;
}
