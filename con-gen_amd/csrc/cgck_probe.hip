// cgck_probe.hip — diagnostics: streaming-read probes that measure the
// practical HBM-read ceiling the checksum kernels are compared with
// (cgck_probe_read).  libcgck.so carries the plain coalesced read (variants
// 0 and 1); the isolation probes behind the measurements of DESIGN.md §5.2
// (block/lane shapes, VALU load, store policies, LDS-DMA reads) are compiled
// only into libcgck_lab.so (-DCGCK_LAB).
#include "cgck_device.h"

namespace cgck {

// --------------------------------------------------------------------------
// Diagnostics: streaming-read probe (what this box's HBM delivers to a plain
// coalesced uint4 read with minimal arithmetic) — the practical ceiling the
// checksum kernels are compared against in DESIGN.md.
// --------------------------------------------------------------------------

template <int UN, bool NT>
__global__ __launch_bounds__(256) void probe_read_kernel(const uint4 *src, uint64_t n16, uint32_t *sink)
{
	uint32_t acc = 0;
	const uint64_t stride = (uint64_t)gridDim.x * 256;
	uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
	for (; i + (UN - 1) * stride < n16; i += UN * stride) {
		uint4 w[UN];
#pragma unroll
		for (int j = 0; j < UN; ++j)
			w[j] = ld<NT>(src + i + j * stride);
#pragma unroll
		for (int j = 0; j < UN; ++j)
			acc = sum4(w[j], acc);
	}
	for (; i < n16; i += stride)
		acc = sum4(src[i], acc);
	if (acc == 0x12345678u) // keeps the loads live; practically never stores
		sink[0] = acc;
}

#if CGCK_LAB
// Contiguous-per-block variant: block b streams [b*per, (b+1)*per).
template <int UN>
__global__ __launch_bounds__(256) void probe_block_kernel(const uint4 *src, uint64_t n16, uint32_t *sink)
{
	uint32_t acc = 0;
	const uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
	const uint64_t b0 = (uint64_t)blockIdx.x * per, b1 = b0 + per < n16 ? b0 + per : n16;
	uint64_t i = b0 + threadIdx.x;
	for (; i + (UN - 1) * 256 < b1; i += UN * 256) {
		uint4 w[UN];
#pragma unroll
		for (int j = 0; j < UN; ++j)
			w[j] = src[i + j * 256];
#pragma unroll
		for (int j = 0; j < UN; ++j)
			acc = sum4(w[j], acc);
	}
	for (; i < b1; i += 256)
		acc = sum4(src[i], acc);
	if (acc == 0x12345678u)
		sink[0] = acc;
}

// Lane-strided variant: lane reads CH consecutive uint4 (one "packet" of
// 16*CH bytes), lanes 16*CH bytes apart — the lane-per-packet access shape.
template <int CH>
__global__ __launch_bounds__(256) void probe_lane_kernel(const uint4 *src, uint64_t n16, uint32_t *sink)
{
	uint32_t acc = 0;
	const uint64_t npk = n16 / CH;
	for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < npk; k += (uint64_t)gridDim.x * 256) {
		uint4 w[CH];
#pragma unroll
		for (int j = 0; j < CH; ++j)
			w[j] = src[k * CH + j];
#pragma unroll
		for (int j = 0; j < CH; ++j)
			acc = sum4(w[j], acc);
	}
	if (acc == 0x12345678u)
		sink[0] = acc;
}

// Latency-structure probe: lane reads 4 uint4 (64 B) per iteration, then
// runs K dependent VALU ops on them; PIPE prefetches the next iteration's
// chunks before the ALU work (software pipelining).
template <int K, bool PIPE>
__global__ __launch_bounds__(256) void probe_alu_kernel(const uint4 *src, uint64_t n16, uint32_t *sink)
{
	uint32_t acc = 0;
	const uint64_t npk = n16 / 4;
	const uint64_t stride = (uint64_t)gridDim.x * 256;
	uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
	uint4 w[4], nx[4];
	if (PIPE && k < npk) {
#pragma unroll
		for (int j = 0; j < 4; ++j)
			nx[j] = src[k * 4 + j];
	}
	for (; k < npk; k += stride) {
#pragma unroll
		for (int j = 0; j < 4; ++j)
			w[j] = PIPE ? nx[j] : src[k * 4 + j];
		if (PIPE && k + stride < npk) {
#pragma unroll
			for (int j = 0; j < 4; ++j)
				nx[j] = src[(k + stride) * 4 + j];
		}
		uint32_t x = 0;
#pragma unroll
		for (int j = 0; j < 4; ++j)
			x = sum4(w[j], x);
#pragma unroll
		for (int i = 0; i < K; ++i)
			x = __builtin_amdgcn_alignbyte(x, x ^ (uint32_t)i, 1u) + (uint32_t)i;
		acc += x;
	}
	if (acc == 0x12345678u)
		sink[0] = acc;
}

// Factor-isolation probe for the 64 B lane-per-packet shape: 4 uint4 per
// lane per iteration, then K dependent VALU, optionally one u32 store per
// lane per iteration (STORE) and an LDS reservation that caps occupancy.
template <int K, bool STORE>
__global__ __launch_bounds__(256) void probe_iso_kernel(const uint4 *src, uint64_t n16, uint32_t *out)
{
	extern __shared__ uint32_t cap[]; // occupancy cap only
	uint32_t acc = 0;
	const uint64_t npk = n16 / 4;
	for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < npk; k += (uint64_t)gridDim.x * 256) {
		uint4 w[4];
#pragma unroll
		for (int j = 0; j < 4; ++j)
			w[j] = ld<false>(src + k * 4 + j);
		uint32_t x = 0;
#pragma unroll
		for (int j = 0; j < 4; ++j)
			x = sum4(w[j], x);
#pragma unroll
		for (int i = 0; i < K; ++i)
			x = __builtin_amdgcn_alignbyte(x, x ^ (uint32_t)i, 1u) + (uint32_t)i;
		if (STORE)
			gbl(out)[k] = x;
		acc += x;
	}
	if (acc == 0x12345678u)
		cap[threadIdx.x] = acc;
}

// Store-shape probes (64 B lane shape): NTS = nontemporal output stores;
// V4 = each lane takes 4 consecutive packets over 4 iterations and writes
// one 16-byte store; CONTIG = block-contiguous packet ranges.
template <bool NTS, bool V4, bool CONTIG>
__global__ __launch_bounds__(256) void probe_store_kernel(const uint4 *src, uint64_t n16, uint32_t *out)
{
	uint32_t acc = 0;
	const uint64_t npk = n16 / 4;
	const uint64_t nit = (npk + 255) / 256;
	const Sched sc = sched(V4 ? (nit + 3) / 4 : nit, CONTIG);
	for (uint64_t it = sc.it; it < sc.end; it += sc.step) {
		if (V4) {
			uint32_t x4[4];
#pragma unroll
			for (int j = 0; j < 4; ++j) {
				const uint64_t k = it * 1024 + threadIdx.x * 4 + j;
				uint4 w[4];
#pragma unroll
				for (int c = 0; c < 4; ++c)
					w[c] = k < npk ? ld<false>(src + k * 4 + c) : make_uint4(0, 0, 0, 0);
				uint32_t x = 0;
#pragma unroll
				for (int c = 0; c < 4; ++c)
					x = sum4(w[c], x);
				x4[j] = x;
			}
			const uint64_t k0 = it * 1024 + threadIdx.x * 4;
			if (k0 + 3 < npk) {
				u32x4_t v = {x4[0], x4[1], x4[2], x4[3]};
				if (NTS)
					__builtin_nontemporal_store(v, (CGCK_GLOBAL u32x4_t *)(out + k0));
				else
					*(CGCK_GLOBAL u32x4_t *)(out + k0) = v;
			}
			acc += x4[0];
		} else {
			const uint64_t k = it * 256 + threadIdx.x;
			if (k >= npk)
				continue;
			uint4 w[4];
#pragma unroll
			for (int c = 0; c < 4; ++c)
				w[c] = ld<false>(src + k * 4 + c);
			uint32_t x = 0;
#pragma unroll
			for (int c = 0; c < 4; ++c)
				x = sum4(w[c], x);
			if (NTS)
				__builtin_nontemporal_store(x, (CGCK_GLOBAL uint32_t *)(out + k));
			else
				gbl(out)[k] = x;
			acc += x;
		}
	}
	if (acc == 0x12345678u)
		out[0] = acc;
}

// Delayed-store probe: iteration i's u32 is stored AFTER iteration i+1's
// loads are issued, so the wait for those loads does not include the store's
// acknowledgement (vmcnt retires in order).
template <int K>
__global__ __launch_bounds__(256) void probe_dstore_kernel(const uint4 *src, uint64_t n16, uint32_t *out)
{
	const uint64_t npk = n16 / 4;
	const uint64_t stride = (uint64_t)gridDim.x * 256;
	uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
	if (k >= npk)
		return;
	uint64_t kprev = k;
	uint32_t xprev = 0;
	for (; k < npk; k += stride) {
		uint4 w[4];
#pragma unroll
		for (int c = 0; c < 4; ++c)
			w[c] = ld<false>(src + k * 4 + c);
		gbl(out)[kprev] = xprev;
		uint32_t x = 0;
#pragma unroll
		for (int c = 0; c < 4; ++c)
			x = sum4(w[c], x);
#pragma unroll
		for (int i = 0; i < K; ++i)
			x = __builtin_amdgcn_alignbyte(x, x ^ (uint32_t)i, 1u) + (uint32_t)i;
		kprev = k;
		xprev = x;
	}
	gbl(out)[kprev] = xprev;
}

// Wave-contiguous 64-B-per-lane reads, 4 x 64 packets per wave step (16
// loads in flight per lane).  MODE 0: u32 store per packet; 1: results
// transposed through LDS, one 16-B store per lane per step; 2: u32 store for
// a quarter of the packets (a quarter of the bytes); 3: no store.
template <int MODE>
__global__ __launch_bounds__(256) void probe_wave4_kernel(const uint4 *src, uint64_t n16, uint32_t *out)
{
	__shared__ uint32_t lds[4][256];
	const uint64_t npk = n16 / 4;
	const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
	const uint64_t nw = (uint64_t)gridDim.x * 4;
	for (uint64_t base = ((uint64_t)blockIdx.x * 4 + wid) * 256; base + 256 <= npk; base += nw * 256) {
		uint4 w[4][4];
#pragma unroll
		for (int j = 0; j < 4; ++j)
#pragma unroll
			for (int c = 0; c < 4; ++c)
				w[j][c] = ld<false>(src + (base + j * 64 + lane) * 4 + c);
		uint32_t r[4];
#pragma unroll
		for (int j = 0; j < 4; ++j) {
			uint32_t x = 0;
#pragma unroll
			for (int c = 0; c < 4; ++c)
				x = sum4(w[j][c], x);
			r[j] = x;
		}
		if (MODE == 0) {
#pragma unroll
			for (int j = 0; j < 4; ++j)
				gbl(out)[base + j * 64 + lane] = r[j];
		} else if (MODE == 1) {
#pragma unroll
			for (int j = 0; j < 4; ++j)
				lds[wid][j * 64 + lane] = r[j];
			__builtin_amdgcn_wave_barrier();
			const u32x4_t v = *reinterpret_cast<const u32x4_t *>(&lds[wid][4 * lane]);
			__builtin_amdgcn_wave_barrier();
			*(CGCK_GLOBAL u32x4_t *)(gbl(out) + base + 4 * lane) = v;
		} else if (MODE == 2) {
			gbl(out)[base / 4 + lane] = r[0] + r[1] + r[2] + r[3];
		} else {
			const uint32_t x = r[0] + r[1] + r[2] + r[3];
			if (x == 0x12345678u)
				gbl(out)[lane] = x;
		}
	}
}

// LDS-DMA streaming probe (MI355X_MICROARCH.md 'ldsdma-fill': 6.4 TB/s
// default policy, 6.5-6.8 nt chip-wide).  One wave per workgroup streams
// its contiguous range through a ring of D 4 KiB slots: 4
// global_load_lds_dwordx4 per slot (1 KiB each, lane l -> bytes 16l), a
// counted vmcnt + s_barrier before the slot is read back with ds_read_b128
// (the RAW rule for LDS-DMA data), and a sum so the data is used.
template <bool NT>
__device__ __forceinline__ void glds16(const void *gsrc, uint32_t lds_dst)
{
	uint32_t keep;
	if (NT)
		asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\t"
			     "s_mov_b32 m0, %0"
			     : "=&s"(keep)
			     : "v"(gsrc), "s"(lds_dst)
			     : "memory");
	else
		asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
			     "s_mov_b32 m0, %0"
			     : "=&s"(keep)
			     : "v"(gsrc), "s"(lds_dst)
			     : "memory");
}

template <int D, bool NT>
__global__ __launch_bounds__(64) void probe_glds_kernel(const uint4 *src, uint64_t n16, uint32_t *sink)
{
	extern __shared__ __attribute__((aligned(16))) uint4 ring[]; // D x 256 uint4
	const int lane = threadIdx.x;
	const uint64_t nst = n16 / 256; // 4 KiB steps
	const uint64_t per = (nst + gridDim.x - 1) / gridDim.x;
	const uint64_t s0 = (uint64_t)blockIdx.x * per, s1 = s0 + per < nst ? s0 + per : nst;
	if (s0 >= s1)
		return;
	const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)ring);
	auto issue = [&](uint64_t st, uint32_t slot) {
		const uint4 *g = src + st * 256 + lane;
#pragma unroll
		for (int j = 0; j < 4; ++j)
			glds16<NT>(g + 64 * j, lds0 + slot * 4096 + 1024 * j);
	};
#pragma unroll
	for (int d = 0; d < D - 1; ++d)
		issue(s0 + d < s1 ? s0 + d : s1 - 1, d);
	uint32_t acc = 0;
	for (uint64_t s = s0; s < s1; ++s) {
		const uint32_t slot = (uint32_t)((s - s0) % D);
		// the slot refilled here was read in the previous step (lgkmcnt(0) below)
		issue(s + D - 1 < s1 ? s + D - 1 : s1 - 1, (uint32_t)((s - s0 + D - 1) % D));
		asm volatile("s_waitcnt vmcnt(%0)" ::"i"((D - 1) * 4) : "memory");
		__builtin_amdgcn_s_barrier();
#pragma unroll
		for (int j = 0; j < 4; ++j)
			acc = sum4(ring[slot * 256 + 64 * j + lane], acc);
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
	}
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	if (acc == 0x12345678u)
		sink[0] = acc;
}

#endif // CGCK_LAB

hipError_t launch_probe_read(const void *src, uint64_t bytes, uint32_t *sink, int num_cus, int variant,
			     hipStream_t st)
{
#if CGCK_LAB
	const uint64_t n16 = bytes / 16;
	const uint4 *sp = reinterpret_cast<const uint4 *>(src);
	const dim3 g(num_cus * 8), b(256);
	switch (variant) {
	case 16: hipLaunchKernelGGL((probe_iso_kernel<0, true>), g, b, 0, st, sp, n16, sink); return hipGetLastError();
	case 17: hipLaunchKernelGGL((probe_iso_kernel<60, false>), g, b, 0, st, sp, n16, sink); return hipGetLastError();
	case 18: hipLaunchKernelGGL((probe_iso_kernel<0, false>), g, b, 32768, st, sp, n16, sink); return hipGetLastError();
	case 19: hipLaunchKernelGGL((probe_iso_kernel<60, true>), g, b, 32768, st, sp, n16, sink); return hipGetLastError();
	case 20: hipLaunchKernelGGL((probe_iso_kernel<60, true>), g, b, 0, st, sp, n16, sink); return hipGetLastError();
	case 21: hipLaunchKernelGGL((probe_iso_kernel<0, true>), g, b, 32768, st, sp, n16, sink); return hipGetLastError();
	case 22: hipLaunchKernelGGL((probe_store_kernel<true, false, false>), g, b, 0, st, sp, n16, sink); return hipGetLastError();
	case 23: hipLaunchKernelGGL((probe_store_kernel<false, true, false>), g, b, 0, st, sp, n16, sink); return hipGetLastError();
	case 24: hipLaunchKernelGGL((probe_store_kernel<true, true, false>), g, b, 0, st, sp, n16, sink); return hipGetLastError();
	case 25: hipLaunchKernelGGL((probe_store_kernel<false, false, true>), g, b, 0, st, sp, n16, sink); return hipGetLastError();
	case 26: hipLaunchKernelGGL((probe_store_kernel<false, true, true>), g, b, 0, st, sp, n16, sink); return hipGetLastError();
	case 27: hipLaunchKernelGGL((probe_store_kernel<true, true, true>), g, b, 0, st, sp, n16, sink); return hipGetLastError();
	case 28: hipLaunchKernelGGL((probe_store_kernel<false, false, false>), g, b, 0, st, sp, n16, sink); return hipGetLastError();
	case 29: hipLaunchKernelGGL((probe_dstore_kernel<0>), g, b, 0, st, sp, n16, sink); return hipGetLastError();
	case 30: hipLaunchKernelGGL((probe_dstore_kernel<60>), g, b, 0, st, sp, n16, sink); return hipGetLastError();
	case 31: hipLaunchKernelGGL((probe_wave4_kernel<0>), g, b, 0, st, sp, n16, sink); return hipGetLastError();
	case 32: hipLaunchKernelGGL((probe_wave4_kernel<1>), g, b, 0, st, sp, n16, sink); return hipGetLastError();
	case 33: hipLaunchKernelGGL((probe_wave4_kernel<2>), g, b, 0, st, sp, n16, sink); return hipGetLastError();
	case 34: hipLaunchKernelGGL((probe_wave4_kernel<3>), g, b, 0, st, sp, n16, sink); return hipGetLastError();
	case 40: hipLaunchKernelGGL((probe_glds_kernel<4, false>), dim3(num_cus * 8), dim3(64), 4 * 4096, st, sp, n16, sink); return hipGetLastError();
	case 41: hipLaunchKernelGGL((probe_glds_kernel<4, true>), dim3(num_cus * 8), dim3(64), 4 * 4096, st, sp, n16, sink); return hipGetLastError();
	case 42: hipLaunchKernelGGL((probe_glds_kernel<8, false>), dim3(num_cus * 4), dim3(64), 8 * 4096, st, sp, n16, sink); return hipGetLastError();
	case 43: hipLaunchKernelGGL((probe_glds_kernel<8, true>), dim3(num_cus * 4), dim3(64), 8 * 4096, st, sp, n16, sink); return hipGetLastError();
	case 44: hipLaunchKernelGGL((probe_glds_kernel<4, true>), dim3(num_cus * 4), dim3(64), 4 * 4096, st, sp, n16, sink); return hipGetLastError();
	case 45: hipLaunchKernelGGL((probe_glds_kernel<8, true>), dim3(num_cus * 8), dim3(64), 8 * 4096, st, sp, n16, sink); return hipGetLastError();
	default: break;
	}
#endif
	const uint4 *s = reinterpret_cast<const uint4 *>(src);
	const uint64_t n = bytes / 16;
	switch (variant) {
	case 1:
		hipLaunchKernelGGL((probe_read_kernel<8, true>), dim3(num_cus * 8), dim3(256), 0, st, s, n, sink);
		break;
#if CGCK_LAB
	case 2:
		hipLaunchKernelGGL((probe_read_kernel<16, false>), dim3(num_cus * 4), dim3(256), 0, st, s, n, sink);
		break;
	case 3:
		hipLaunchKernelGGL((probe_read_kernel<4, false>), dim3(num_cus * 16), dim3(256), 0, st, s, n, sink);
		break;
	case 4:
		hipLaunchKernelGGL((probe_block_kernel<8>), dim3(num_cus * 8), dim3(256), 0, st, s, n, sink);
		break;
	case 5:
		hipLaunchKernelGGL((probe_read_kernel<8, false>), dim3(num_cus * 32), dim3(256), 0, st, s, n, sink);
		break;
	case 6:
		hipLaunchKernelGGL((probe_lane_kernel<4>), dim3(num_cus * 8), dim3(256), 0, st, s, n, sink);
		break;
	case 7:
		hipLaunchKernelGGL((probe_lane_kernel<8>), dim3(num_cus * 8), dim3(256), 0, st, s, n, sink);
		break;
	case 8:
		hipLaunchKernelGGL((probe_lane_kernel<2>), dim3(num_cus * 8), dim3(256), 0, st, s, n, sink);
		break;
	case 9:
		hipLaunchKernelGGL((probe_alu_kernel<100, false>), dim3(num_cus * 8), dim3(256), 0, st, s, n, sink);
		break;
	case 10:
		hipLaunchKernelGGL((probe_alu_kernel<300, false>), dim3(num_cus * 8), dim3(256), 0, st, s, n, sink);
		break;
	case 11:
		hipLaunchKernelGGL((probe_alu_kernel<600, false>), dim3(num_cus * 8), dim3(256), 0, st, s, n, sink);
		break;
	case 12:
		hipLaunchKernelGGL((probe_alu_kernel<100, true>), dim3(num_cus * 8), dim3(256), 0, st, s, n, sink);
		break;
	case 13:
		hipLaunchKernelGGL((probe_alu_kernel<300, true>), dim3(num_cus * 8), dim3(256), 0, st, s, n, sink);
		break;
	case 14:
		hipLaunchKernelGGL((probe_alu_kernel<600, true>), dim3(num_cus * 8), dim3(256), 0, st, s, n, sink);
		break;
	case 15:
		hipLaunchKernelGGL((probe_alu_kernel<0, false>), dim3(num_cus * 8), dim3(256), 0, st, s, n, sink);
		break;
#endif
	default:
		hipLaunchKernelGGL((probe_read_kernel<8, false>), dim3(num_cus * 8), dim3(256), 0, st, s, n, sink);
	}
	return hipGetLastError();
}

} // namespace cgck
