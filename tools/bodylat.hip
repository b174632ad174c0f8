// bodylat.hip — what does the burst server's body cost for one small
// request, and where?  ("2.3 us of compute for one 64 B
// packet is ~5,500 cycles at 2.39 GHz".)  Not product code: a standalone
// probe (make -C tools bodylat) that compiles the server's own body
// (cgck_group.hip's burst_body, the one-workgroup LDS-resident path) into a
// kernel of its own, runs it `reps` times back to back on a request block
// held in LDS, and reports the shader-clock cycles of each run (s_memtime
// around the body and the barrier after it, as the server's lab timers).
//
//   bodylat [npkts] [len] [raw|verify|fill] [reps] [spec]
//
// One JSON line: median / p10 / p90 cycles, and the outputs of packet 0 for
// a sanity check against the host's own sum.
#include "../con-gen_amd/csrc/cgck_group.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <algorithm>

using namespace cgck;

// the library's launch bookkeeping, which the included file's launchers name
namespace cgck {
thread_local const char *t_kernel;
const char *intern(const char *fmt, ...) { return fmt; }
} // namespace cgck

#define CHECK(x)                                                                          \
	do {                                                                              \
		hipError_t e_ = (x);                                                      \
		if (e_ != hipSuccess) {                                                   \
			fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
			exit(1);                                                          \
		}                                                                         \
	} while (0)

// LIVE: uniform values kept live across the body (the server kernel's state
// around its body: its arguments, loop and request words), the A/B of
// "bodylat ... live"
struct LiveArgs {
	uint64_t v[20];
};

template <uint32_t FL, bool LIVE = false>
__global__ __launch_bounds__(256) void bodylat_kernel(const uint8_t *blk, uint32_t *out, uint32_t *meta, uint8_t *ver,
						       uint64_t *ticks, int reps, LiveArgs la = {})
{
	__shared__ uint4 hdr_w[4];
	__shared__ uint4 sblock[kBurstFirst / 16];
	__shared__ uint4 szero;
	const int t = threadIdx.x;
	if (t == 0)
		szero = make_uint4(0, 0, 0, 0);
	const uint4 *src = reinterpret_cast<const uint4 *>(blk);
	const uint4 v0 = src[t], v1 = src[256 + t];
	if (t < 4)
		hdr_w[t] = v0;
	sblock[t] = v0;
	sblock[256 + t] = v1;
	__syncthreads();
	const BurstReq &h = *reinterpret_cast<const BurstReq *>(hdr_w);
	const uint32_t n = h.n;
	const uint32_t *sd = reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(sblock) + sizeof(BurstReq));
	const uint8_t *base = reinterpret_cast<const uint8_t *>(sblock) + h.p_off;
	for (int r = 0; r < reps; ++r) {
		__syncthreads();
		const uint64_t c0 = __builtin_amdgcn_s_memtime();
		uint64_t lv[20];
		if constexpr (LIVE) {
#pragma unroll
			for (int i = 0; i < 20; ++i)
				lv[i] = la.v[i] * (uint64_t)(r + 1); // uniform, defined before the body
		}
		burst_body<true, false, true, true, FL>(h, sd, 0, n, out, meta, ver, &szero, base);
		__syncthreads();
		const uint64_t c1 = __builtin_amdgcn_s_memtime();
		if (t == 0)
			ticks[r] = c1 - c0;
		if constexpr (LIVE) { // ... and used after it
			uint64_t x = 0;
#pragma unroll
			for (int i = 0; i < 20; ++i)
				x ^= lv[i] >> (i & 7);
			if (t == 0 && x == 0x123456789ull)
				ticks[reps] = x;
		}
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	}
}

int main(int argc, char **argv)
{
	const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 1;
	const uint32_t len = argc > 2 ? (uint32_t)atoi(argv[2]) : 64;
	const char *mode = argc > 3 ? argv[3] : "verify";
	const int reps = argc > 4 ? atoi(argv[4]) : 2000;
	const uint32_t flags = !strcmp(mode, "raw")    ? CGCK_RAW
			       : !strcmp(mode, "fill") ? CGCK_IP | CGCK_L4 | CGCK_ZERO_FIELDS
						       : CGCK_IP | CGCK_L4 | CGCK_VERIFY | CGCK_V_IP_ZERO_IS_FFFF |
							 CGCK_V_UDP_ZERO_SKIP;
	const uint32_t d_off = sizeof(BurstReq), p_off = (d_off + 12 * n + 15) & ~15u;
	const uint32_t bytes = p_off + n * len;
	if (n == 0 || len < 20 || bytes > kBurstFirst) {
		fprintf(stderr, "bodylat: the block must fit %u bytes\n", kBurstFirst);
		return 2;
	}
	std::vector<uint8_t> b(kBurstFirst, 0);
	BurstReq hq;
	memset(&hq, 0, sizeof(hq));
	hq.n = n;
	hq.flags = flags;
	hq.max_len = len;
	hq.bytes = bytes;
	hq.d_off = d_off;
	hq.p_off = p_off;
	memcpy(b.data(), &hq, sizeof(hq));
	for (uint32_t i = 0; i < n; i++) {
		uint32_t d[3] = {i * len, 0, len << 16};
		memcpy(b.data() + d_off + 12 * i, d, 12);
		uint8_t *ip = b.data() + p_off + i * len;
		for (uint32_t k = 0; k < len; k++)
			ip[k] = (uint8_t)(i * 7 + k * 13);
		ip[0] = 0x45;
		ip[2] = (uint8_t)(len >> 8);
		ip[3] = (uint8_t)len;
		ip[9] = 17;
	}
	uint8_t *blk;
	uint32_t *out, *meta;
	uint8_t *ver;
	uint64_t *ticks;
	CHECK(hipMalloc((void **)&blk, kBurstFirst));
	CHECK(hipMemcpy(blk, b.data(), kBurstFirst, hipMemcpyHostToDevice));
	// outputs in host-coherent memory, as the server's
	CHECK(hipHostMalloc((void **)&out, 4 * 64 + 64, hipHostMallocCoherent));
	CHECK(hipHostMalloc((void **)&meta, 4 * 64 + 64, hipHostMallocCoherent));
	CHECK(hipHostMalloc((void **)&ver, 64 + 64, hipHostMallocCoherent));
	CHECK(hipMalloc((void **)&ticks, sizeof(uint64_t) * (reps + 1)));
	// argv[5] "spec": the body compiled for these flags (FL), else read at run time;
	// "live": the BSD verify body with 20 uniform 64-bit values live across it
	const bool spec = argc > 5 && !strcmp(argv[5], "spec");
	const bool live = argc > 5 && !strcmp(argv[5], "live");
	LiveArgs la;
	for (int i = 0; i < 20; i++)
		la.v[i] = 0x9E3779B97F4A7C15ull * (uint64_t)(i + 1);
	if (live && flags == CGCK_RAW)
		hipLaunchKernelGGL((bodylat_kernel<CGCK_RAW, true>), dim3(1), dim3(256), 0, 0, blk, out, meta, ver, ticks,
				   reps, la);
	else if (live)
		hipLaunchKernelGGL((bodylat_kernel<CGCK_VERIFY_BSD, true>), dim3(1), dim3(256), 0, 0, blk, out, meta, ver,
				   ticks, reps, la);
	else if (!spec)
		hipLaunchKernelGGL(bodylat_kernel<0>, dim3(1), dim3(256), 0, 0, blk, out, meta, ver, ticks, reps);
	else if (flags == CGCK_RAW)
		hipLaunchKernelGGL(bodylat_kernel<CGCK_RAW>, dim3(1), dim3(256), 0, 0, blk, out, meta, ver, ticks, reps);
	else if (flags == (CGCK_IP | CGCK_L4 | CGCK_ZERO_FIELDS))
		hipLaunchKernelGGL(bodylat_kernel<CGCK_IP | CGCK_L4 | CGCK_ZERO_FIELDS>, dim3(1), dim3(256), 0, 0, blk, out,
				   meta, ver, ticks, reps);
	else
		hipLaunchKernelGGL(bodylat_kernel<CGCK_VERIFY_BSD>, dim3(1), dim3(256), 0, 0, blk, out, meta, ver, ticks,
				   reps);
	CHECK(hipGetLastError());
	CHECK(hipDeviceSynchronize());
	std::vector<uint64_t> tk(reps);
	CHECK(hipMemcpy(tk.data(), ticks, sizeof(uint64_t) * reps, hipMemcpyDeviceToHost));
	std::sort(tk.begin(), tk.end());
	// the host's own one's-complement sum of packet 0 (raw) for a sanity check
	uint32_t s = 0;
	const uint8_t *ip = b.data() + p_off;
	for (uint32_t k = 0; k + 1 < len; k += 2)
		s += ip[k] | ip[k + 1] << 8;
	if (len & 1)
		s += ip[len - 1];
	while (s >> 16)
		s = (s & 0xffff) + (s >> 16);
	printf("{\"npkts\": %u, \"len\": %u, \"mode\": \"%s\", \"spec\": %d, \"live\": %d, \"reps\": %d, \"cycles_median\": %llu, \"cycles_p10\": %llu, "
	       "\"cycles_p90\": %llu, \"out0\": \"0x%08x\", \"ver0\": %u, \"host_raw0\": \"0x%04x\"}\n",
	       n, len, mode, (int)spec, (int)live, reps, (unsigned long long)tk[reps / 2], (unsigned long long)tk[reps / 10],
	       (unsigned long long)tk[reps * 9 / 10], out[0], ver[0], (~s) & 0xffff);
	return 0;
}
