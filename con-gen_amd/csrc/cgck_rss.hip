// cgck_rss.hip — gfx950 kernels for con-gen's Toeplitz RSS hash
// (toeplitz_hash / rss_hash4, subr.c:482-530) and for the dst-cache build
// that calls it once per candidate 4-tuple (thread_init_dst_cache,
// con-gen.c:291-360).  SURVEY §8(f) rank 4.
//
// Arithmetic.  toeplitz_hash() shifts a 32-bit window along the key bit
// stream and XORs it into h for every set data bit.  With W(p) = the 32 key
// bits starting at bit p (MSB first; the reference reads key[0..3] and then
// key[4..key_size-1], zeros after), h = XOR over set data bits p of W(p).
// That is linear over GF(2), so the bits of one data byte fold into a table
// T[i][v] = XOR of W(8i+b) over the set bits b of v (built on the host,
// cgck_api.cpp).  A tuple then costs one LDS lookup and one XOR per byte:
// 12 for the IPv4 4-tuple of rss_hash4.  Bit-exact by construction.
//
// Both kernels are integer work with no GEMM shape.  The batched hash is
// HBM-bound (12 B read + 4 B written per tuple); the dst-cache build reads
// nothing (it enumerates its tuples) and is bound by VALU/LDS issue.
#include "cgck_device.h"

#include <stdlib.h>

namespace cgck {

#define RLX_AGENT __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT

// ---------------------------------------------------------------------------
// Batched hash: out[k] = toeplitz_hash(data + k*stride, cnt, key) & mask
// ---------------------------------------------------------------------------

// CW > 0: records are cnt = 4*CW bytes, dword aligned (the IPv4 4-tuple is
// CW = 3, the IPv6 one CW = 9): CW dword loads per lane.  CW = 0: any cnt,
// byte loads.  LDS: the cnt x 256 table is staged in LDS (cnt <= 36), else
// read from global memory (L2-resident).
template <int CW, bool LDS>
__global__ __launch_bounds__(256) void toeplitz_kernel(RssParams p)
{
	extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
	const uint32_t CGCK_GLOBAL *gt = (const uint32_t CGCK_GLOBAL *)p.tab;
	if (LDS) {
		const uint32_t tn = p.cnt * 256;
		for (uint32_t i = threadIdx.x; i < tn; i += 256)
			smem[i] = gt[i];
		__syncthreads();
	}
	const uint8_t CGCK_GLOBAL *data = (const uint8_t CGCK_GLOBAL *)p.data;
	uint32_t CGCK_GLOBAL *out = (uint32_t CGCK_GLOBAL *)p.out;
	const uint64_t step = (uint64_t)gridDim.x * 256;
	for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < p.n; k += step) {
		const uint8_t CGCK_GLOBAL *r = data + k * p.stride;
		uint32_t h = 0;
		if (CW > 0) {
			const uint32_t CGCK_GLOBAL *rw = (const uint32_t CGCK_GLOBAL *)r;
			uint32_t w[CW > 0 ? CW : 1];
#pragma unroll
			for (int c = 0; c < CW; c++)
				w[c] = rw[c];
#pragma unroll
			for (int c = 0; c < CW; c++)
#pragma unroll
				for (int j = 0; j < 4; j++) {
					const uint32_t v = (w[c] >> (8 * j)) & 255u;
					h ^= LDS ? smem[(4 * c + j) * 256 + v] : gt[(4 * c + j) * 256 + v];
				}
		} else {
			for (uint32_t i = 0; i < p.cnt; i++) {
				const uint32_t v = r[i];
				h ^= LDS ? smem[i * 256 + v] : gt[i * 256 + v];
			}
		}
		out[k] = h & p.mask;
	}
}

// Dense 12-byte records (the rss_hash4 tuple array), 16-byte aligned: each
// lane takes 4 consecutive records = 48 bytes = 3 uint4 loads, and writes
// its 4 results as one uint4 (16 B per lane, coalesced).  Two groups per
// lane are loaded before either is hashed, so 6 loads are in flight.
// Byte tables: 12 ds_read_b32 per tuple, but 32 lanes of random bytes land
// on the 32 banks with ~3.5-way conflicts (MI355X_MICROARCH.md § LDS).
// Nibble tables (NIB): 24 lookups into 16-entry rows, which map onto 16
// distinct banks, so every access pattern is conflict-free (identical
// addresses broadcast).  NT[2i][v] = T[i][v << 4] (high nibble of byte i),
// NT[2i+1][v] = T[i][v].
template <bool NIB>
__device__ __forceinline__ uint32_t hash12(const uint32_t *T, uint32_t w0, uint32_t w1, uint32_t w2)
{
	uint32_t h = 0;
	const uint32_t w[3] = {w0, w1, w2};
#pragma unroll
	for (int c = 0; c < 3; c++)
#pragma unroll
		for (int j = 0; j < 4; j++) {
			if (NIB) {
				h ^= T[(2 * (4 * c + j) + 0) * 16 + ((w[c] >> (8 * j + 4)) & 15u)];
				h ^= T[(2 * (4 * c + j) + 1) * 16 + ((w[c] >> (8 * j)) & 15u)];
			} else {
				h ^= T[(4 * c + j) * 256 + ((w[c] >> (8 * j)) & 255u)];
			}
		}
	return h;
}

template <bool NIB>
__device__ __forceinline__ u32x4_t hash4x12(const uint32_t *T, const u32x4_t &a, const u32x4_t &b,
					    const u32x4_t &c, uint32_t mask)
{
	u32x4_t o;
	o.x = hash12<NIB>(T, a.x, a.y, a.z) & mask;
	o.y = hash12<NIB>(T, a.w, b.x, b.y) & mask;
	o.z = hash12<NIB>(T, b.z, b.w, c.x) & mask;
	o.w = hash12<NIB>(T, c.y, c.z, c.w) & mask;
	return o;
}

template <bool NIB>
__global__ __launch_bounds__(256) void toeplitz12x4_kernel(RssParams p, uint64_t ng)
{
	extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
	const uint32_t CGCK_GLOBAL *gt = (const uint32_t CGCK_GLOBAL *)p.tab;
	if (NIB) {
		for (uint32_t i = threadIdx.x; i < 24 * 16; i += 256) {
			const uint32_t r = i >> 4, v = i & 15;
			smem[i] = gt[(r >> 1) * 256 + ((r & 1) ? v : v << 4)];
		}
	} else {
		for (uint32_t i = threadIdx.x; i < 12 * 256; i += 256)
			smem[i] = gt[i];
	}
	__syncthreads();
	const u32x4_t CGCK_GLOBAL *src = (const u32x4_t CGCK_GLOBAL *)p.data;
	u32x4_t CGCK_GLOBAL *out = (u32x4_t CGCK_GLOBAL *)p.out;
	const uint64_t step = (uint64_t)gridDim.x * 256;
	uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
	for (; g + step < ng; g += 2 * step) {
		const uint64_t g2 = g + step;
		const u32x4_t a0 = src[3 * g], b0 = src[3 * g + 1], c0 = src[3 * g + 2];
		const u32x4_t a1 = src[3 * g2], b1 = src[3 * g2 + 1], c1 = src[3 * g2 + 2];
		out[g] = hash4x12<NIB>(smem, a0, b0, c0, p.mask);
		out[g2] = hash4x12<NIB>(smem, a1, b1, c1, p.mask);
	}
	if (g < ng) {
		const u32x4_t a = src[3 * g], b = src[3 * g + 1], c = src[3 * g + 2];
		out[g] = hash4x12<NIB>(smem, a, b, c, p.mask);
	}
}

// Software-pipelined form (the lpa lesson, cgck_lane.hip): per lane DEPTH
// 48-byte groups in flight in a register ring, loads unconditional
// (index clamped to the last group), so each group's output store trails the
// next group's loads and no wait includes a store acknowledgement; the store
// is inline asm so the compiler does not hold later registers behind it.
// Nontemporal store: +1.8 % in one process against the plain store
// (tools/ab_inproc.py, profiles/r01/ab_rss_nt.log; 64 B control 0.998).
__device__ __forceinline__ void t12_load(const u32x4_t CGCK_GLOBAL *src, uint64_t g, uint64_t ng, u32x4_t (&r)[3])
{
	const uint64_t gg = g < ng ? g : ng - 1;
	r[0] = src[3 * gg];
	r[1] = src[3 * gg + 1];
	r[2] = src[3 * gg + 2];
}

__device__ __forceinline__ void t12_store(uint32_t *out, uint64_t g, const u32x4_t &v)
{
	u32x4_t *o = reinterpret_cast<u32x4_t *>(out) + g;
	asm volatile("global_store_dwordx4 %0, %1, off nt\n\ts_nop 1" ::"v"(o), "v"(v) : "memory");
}

template <int DEPTH>
__global__ __launch_bounds__(256) void toeplitz12x4_ab_kernel(RssParams p, uint64_t ng)
{
	extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
	const uint32_t CGCK_GLOBAL *gt = (const uint32_t CGCK_GLOBAL *)p.tab;
	for (uint32_t i = threadIdx.x; i < 12 * 256; i += 256)
		smem[i] = gt[i];
	__syncthreads();
	const u32x4_t CGCK_GLOBAL *src = (const u32x4_t CGCK_GLOBAL *)p.data;
	const uint64_t NI = (ng + 255) / 256, S = gridDim.x;
	uint64_t it = blockIdx.x;
	if (it >= NI)
		return;
	// DEPTH groups per lane in a register ring: group d + DEPTH - 1 is loaded
	// before group d is hashed (past the end the index clamps to this block's
	// last group, so no load sits under a branch)
	auto gof = [&](uint64_t i) { return (i < NI ? i : it) * 256 + threadIdx.x; };
	u32x4_t R[DEPTH][3];
#pragma unroll
	for (int d = 0; d < DEPTH - 1; ++d)
		t12_load(src, gof(it + d * S), ng, R[d]);
	for (;;) {
#pragma unroll
		for (int d = 0; d < DEPTH; ++d) {
			t12_load(src, gof(it + (uint64_t)(d + DEPTH - 1) * S), ng, R[(d + DEPTH - 1) % DEPTH]);
			const uint64_t g = (it + d * S) * 256 + threadIdx.x;
			const u32x4_t h = hash4x12<false>(smem, R[d][0], R[d][1], R[d][2], p.mask);
			if (g < ng)
				t12_store(p.out, g, h);
			if (it + (uint64_t)(d + 1) * S >= NI)
				return;
		}
		it += (uint64_t)DEPTH * S;
	}
}

// 12-bit tables.  The record's 96 bits, read as one little-endian integer X
// (dwords w0 w1 w2), split into eight 12-bit fields f = (X >> 12k) & 0xfff, so
// a tuple costs 8 LDS lookups instead of 12.  T12[k][v] comes from the byte
// tables by linearity: an even field 2m is byte 3m and the low nibble of byte
// 3m + 1, an odd field 2m + 1 the high nibble of byte 3m + 1 and byte 3m + 2.
// The eight tables take 128 KiB of LDS: one workgroup per CU, up to 16 waves.
__device__ __forceinline__ uint32_t hash12_t12(const uint32_t *T, uint32_t w0, uint32_t w1, uint32_t w2)
{
	const uint32_t f2 = __builtin_amdgcn_alignbit(w1, w0, 24), f5 = __builtin_amdgcn_alignbit(w2, w1, 28);
	return T[w0 & 0xfffu] ^ T[4096 + ((w0 >> 12) & 0xfffu)] ^ T[2 * 4096 + (f2 & 0xfffu)] ^
	       T[3 * 4096 + ((w1 >> 4) & 0xfffu)] ^ T[4 * 4096 + ((w1 >> 16) & 0xfffu)] ^
	       T[5 * 4096 + (f5 & 0xfffu)] ^ T[6 * 4096 + ((w2 >> 8) & 0xfffu)] ^ T[7 * 4096 + (w2 >> 20)];
}

constexpr uint32_t kT12Words = 8 * 4096;

template <int DEPTH, int TPB>
__global__ __launch_bounds__(TPB) void toeplitz12x4_t12_kernel(RssParams p, uint64_t ng)
{
	__shared__ __attribute__((aligned(16))) uint32_t smem[kT12Words + 12 * 256];
	uint32_t *t8 = smem + kT12Words;
	const uint32_t CGCK_GLOBAL *gt = (const uint32_t CGCK_GLOBAL *)p.tab;
	for (uint32_t i = threadIdx.x; i < 12 * 256; i += TPB)
		t8[i] = gt[i];
	__syncthreads();
	for (uint32_t e = threadIdx.x; e < kT12Words; e += TPB) {
		const uint32_t k = e >> 12, v = e & 4095u, m = k >> 1;
		smem[e] = (k & 1) ? t8[(3 * m + 1) * 256 + ((v & 15u) << 4)] ^ t8[(3 * m + 2) * 256 + (v >> 4)]
				  : t8[3 * m * 256 + (v & 255u)] ^ t8[(3 * m + 1) * 256 + ((v >> 8) & 15u)];
	}
	__syncthreads();
	const u32x4_t CGCK_GLOBAL *src = (const u32x4_t CGCK_GLOBAL *)p.data;
	const uint64_t NI = (ng + TPB - 1) / TPB, S = gridDim.x;
	uint64_t it = blockIdx.x;
	if (it >= NI)
		return;
	// the register ring of toeplitz12x4_ab_kernel, TPB groups per block step
	auto gof = [&](uint64_t i) { return (i < NI ? i : it) * TPB + threadIdx.x; };
	u32x4_t R[DEPTH][3];
#pragma unroll
	for (int d = 0; d < DEPTH - 1; ++d)
		t12_load(src, gof(it + d * S), ng, R[d]);
	for (;;) {
#pragma unroll
		for (int d = 0; d < DEPTH; ++d) {
			t12_load(src, gof(it + (uint64_t)(d + DEPTH - 1) * S), ng, R[(d + DEPTH - 1) % DEPTH]);
			const uint64_t g = (it + d * S) * TPB + threadIdx.x;
			u32x4_t h;
			h.x = hash12_t12(smem, R[d][0].x, R[d][0].y, R[d][0].z) & p.mask;
			h.y = hash12_t12(smem, R[d][0].w, R[d][1].x, R[d][1].y) & p.mask;
			h.z = hash12_t12(smem, R[d][1].z, R[d][1].w, R[d][2].x) & p.mask;
			h.w = hash12_t12(smem, R[d][2].y, R[d][2].z, R[d][2].w) & p.mask;
			if (g < ng)
				t12_store(p.out, g, h);
			if (it + (uint64_t)(d + 1) * S >= NI)
				return;
		}
		it += (uint64_t)DEPTH * S;
	}
}

hipError_t launch_toeplitz(const RssParams &p0, int num_cus, hipStream_t st)
{
	if (p0.n == 0)
		return hipSuccess;
	RssParams p = p0;
	if (p.cnt == 12 && p.stride == 12 && ((uintptr_t)p.data & 15) == 0 && ((uintptr_t)p.out & 15) == 0 &&
	    p.n >= 4) {
		const uint64_t ng = p.n / 4;
		const uint64_t want = (ng + 255) / 256;
		// Byte tables: measured 0.225 vs 0.233 ms for nibble tables on 64M
		// tuples (the kernel is bound by the mixed read/write stream, not by
		// LDS conflicts).
		static const int var = [] { // $CGCK_RSS_VAR: 0 two-group loop, 1 nibble tables, 2 A/B pipelined
			const char *e = CGCK_ENV("CGCK_RSS_VAR");
			return e ? atoi(e) : kDefaultRssVariant;
		}();
		// 1 block per CU with a deep register ring (below); at the earlier
		// depth 3, 2 blocks per CU read 65.4 % of HBM peak vs 62.5 % at 8
		// (tools/rss_sweep.sh)
		static const int bpc = [] {
			const char *e = CGCK_ENV("CGCK_RSS_BPC");
			return e && atoi(e) > 0 ? atoi(e) : 1;
		}();
		// ring depth 12 at 1 block per CU (181 VGPRs, no spills), in-process
		// A/B chain (tools/ab_inproc.py, profiles/r01/ab_rss_depth_chain.log):
		// depth 3 at 2 blocks/CU -> depth 4 at 1 block +1.7 %, 5 +3.1 %, 6 +4.6 %
		// over 4; 8 +1.2 %, 10 +3.6 % over 6; 12 +2.9 %, 16 -1.7 % over 10
		// (76.7 % of peak); 2 blocks/CU at depth 6 -8 %
		static const int depth = [] { // $CGCK_RSS_DEPTH: groups per lane in flight, 2..6, 8, 10, 12, 16
			const char *e = CGCK_ENV("CGCK_RSS_DEPTH");
			const int d = e ? atoi(e) : 0;
			return (d >= 2 && d <= 6) || d == 8 || d == 10 || d == 12 || d == 16 ? d : 12;
		}();
		const uint64_t capb = (uint64_t)num_cus * bpc;
		const dim3 gb((unsigned)(want < capb ? want : capb));
#define CGCK_RSS_AB(D)                                                                          \
	do {                                                                                    \
		CGCK_NOTE_KERNEL("toeplitz12x4_ab_kernel<%d>", D);                              \
		hipLaunchKernelGGL(toeplitz12x4_ab_kernel<D>, gb, dim3(256), 12 * 256 * 4, st, p, ng); \
	} while (0)
#if CGCK_LAB
		// var 3: 12-bit tables, $CGCK_RSS_TPB threads (256 | 512 | 1024), one workgroup per CU
		static const int tpb = [] {
			const char *e = CGCK_ENV("CGCK_RSS_TPB");
			const int t = e ? atoi(e) : 512;
			return t == 256 || t == 1024 ? t : 512;
		}();
#define CGCK_RSS_T12(D, T)                                                                              \
	if (depth == D && tpb == T) {                                                                   \
		const uint64_t wt = (ng + T - 1) / T;                                                   \
		const dim3 gt((unsigned)(wt < (uint64_t)num_cus ? wt : (uint64_t)num_cus));             \
		CGCK_NOTE_KERNEL("toeplitz12x4_t12_kernel<%d, %d>", D, T);                               \
		hipLaunchKernelGGL((toeplitz12x4_t12_kernel<D, T>), gt, dim3(T), 0, st, p, ng);          \
	} else
		if (var == 3) {
			CGCK_RSS_T12(2, 1024) CGCK_RSS_T12(3, 1024) CGCK_RSS_T12(4, 512) CGCK_RSS_T12(6, 512)
			CGCK_RSS_T12(8, 512) CGCK_RSS_T12(4, 256) CGCK_RSS_T12(8, 256) CGCK_RSS_T12(12, 256)
			CGCK_RSS_T12(4, 1024) CGCK_RSS_AB(12);
		} else if (var == 2 && depth == 16)
			CGCK_RSS_AB(16);
		else if (var == 2 && depth == 12)
			CGCK_RSS_AB(12);
		else if (var == 2 && depth == 10)
			CGCK_RSS_AB(10);
		else if (var == 2 && depth == 8)
			CGCK_RSS_AB(8);
		else if (var == 2 && depth == 6)
			CGCK_RSS_AB(6);
		else if (var == 2 && depth == 5)
			CGCK_RSS_AB(5);
		else if (var == 2 && depth == 4)
			CGCK_RSS_AB(4);
		else if (var == 2 && depth == 3)
			CGCK_RSS_AB(3);
		else if (var == 2)
			CGCK_RSS_AB(2);
		else if (var == 1) {
			CGCK_NOTE_KERNEL("toeplitz12x4_kernel<true>");
			hipLaunchKernelGGL(toeplitz12x4_kernel<true>, gb, dim3(256), 24 * 16 * 4, st, p, ng);
		} else {
			CGCK_NOTE_KERNEL("toeplitz12x4_kernel<false>");
			hipLaunchKernelGGL(toeplitz12x4_kernel<false>, gb, dim3(256), 12 * 256 * 4, st, p, ng);
		}
#else
		(void)var;
		(void)depth;
		CGCK_RSS_AB(12); // the measured default; the other depths and forms are lab builds
#endif
#undef CGCK_RSS_AB
#if CGCK_LAB
#undef CGCK_RSS_T12
#endif
		hipError_t e = hipGetLastError();
		if (e != hipSuccess || ng * 4 == p.n)
			return e;
		p.data += ng * 48;
		p.out += ng * 4;
		p.n -= ng * 4;
	}
	const uint64_t want = (p.n + 255) / 256;
	const uint64_t cap = (uint64_t)num_cus * 8;
	const dim3 g((unsigned)(want < cap ? want : cap)), b(256);
	const bool aligned = ((uintptr_t)p.data & 3) == 0 && (p.stride & 3) == 0;
	const bool lds = p.cnt <= kRssLdsMaxCnt;
	const size_t sh = lds ? (size_t)p.cnt * 256 * 4 : 0;
	// (after the x4 kernel this is the n % 4 tail: the x4 kernel keeps the name)
	const bool note = p.n == p0.n;
	if (aligned && p.cnt == 12) {
		if (note)
			CGCK_NOTE_KERNEL("toeplitz_kernel<3, true>");
		hipLaunchKernelGGL((toeplitz_kernel<3, true>), g, b, sh, st, p);
	} else if (aligned && p.cnt == 36) {
		if (note)
			CGCK_NOTE_KERNEL("toeplitz_kernel<9, true>");
		hipLaunchKernelGGL((toeplitz_kernel<9, true>), g, b, sh, st, p);
	} else if (lds) {
		if (note)
			CGCK_NOTE_KERNEL("toeplitz_kernel<0, true>");
		hipLaunchKernelGGL((toeplitz_kernel<0, true>), g, b, sh, st, p);
	} else {
		if (note)
			CGCK_NOTE_KERNEL("toeplitz_kernel<0, false>");
		hipLaunchKernelGGL((toeplitz_kernel<0, false>), g, b, 0, st, p);
	}
	return hipGetLastError();
}

// ---------------------------------------------------------------------------
// dst-cache build (con-gen.c:291-360)
// ---------------------------------------------------------------------------
//
// Tuple i of the reference loop is the mixed-radix decomposition of i:
// faddr fastest (faddr_min + i % nf), then the ephemeral local port
// (5000 + (i / nf) % 60536), then laddr (laddr_min + i / (nf * 60536)):
// con-gen.c:320-333 advances exactly that way and never wraps for i < n.
// Survivors of the RSS filter (con-gen.c:337-342) are written in loop order
// until `cap` of them exist (con-gen.c:344-353).
//
// One persistent launch.  Workgroups draw 4096-tuple tiles from a ticket
// counter; each tile takes its output offset from the tiles before it by a
// decoupled look-back (every tile publishes its count as an AGG word, then
// its inclusive prefix as an INCL word; one wave sums predecessors 64 at a
// time until it meets an INCL).  The status words carry their own flag, so
// they are the only cross-workgroup data (Guideline 16, form R2: 8-byte
// relaxed agent-scope atomics, no fence).  Tickets are drawn in order and a
// tile always publishes, so every look-back ends; the spin is bounded anyway
// and reports a timeout.  Once a tile's prefix reaches `cap` no new tickets
// are drawn.

constexpr int kDstWaves = 4, kDstIters = 512; // iterations per wave per tile: p.iters <= kDstIters
constexpr uint32_t kNEph = 65535 - 5000 + 1;             // NEPHEMERAL (subr.h:62-64)
constexpr uint32_t kEphMin = 5000;                        // EPHEMERAL_MIN
constexpr uint64_t kStAgg = 1ull << 62, kStIncl = 2ull << 62;
constexpr uint32_t kSpinLimit = 1u << 22;
constexpr int kLookWin = 4; // predecessor words per lane per look-back round trip (256 per wave)

// LDS carve-up (dynamic, 16-byte aligned; Guideline 17): [tables 12 KiB when
// filtering] [survivor bits: waves x iters/32 x 64 u32] [S: 16 u32].
constexpr uint32_t kDstMaskBytes = kDstWaves * (kDstIters / 32) * 64 * 4;

// Per-lane tuple cursor: offsets into the faddr, lport and laddr ranges,
// and the hash share of the laddr bytes and fport (recomputed only when
// laddr changes, once per 60536 x nf tuples).  The faddr and lport shares
// are looked up per tuple, unconditionally, so the loop has no divergent
// branch on the common path.
struct Cursor {
	uint32_t fa, lp, la;
	uint32_t hl;
};

__device__ __forceinline__ uint32_t hash_fa(const uint32_t *T, uint32_t fa)
{
	return T[0 * 256 + (fa >> 24)] ^ T[1 * 256 + ((fa >> 16) & 255u)] ^ T[2 * 256 + ((fa >> 8) & 255u)] ^
	       T[3 * 256 + (fa & 255u)];
}

__device__ __forceinline__ uint32_t hash_la(const uint32_t *T, uint32_t la)
{
	return T[4 * 256 + (la >> 24)] ^ T[5 * 256 + ((la >> 16) & 255u)] ^ T[6 * 256 + ((la >> 8) & 255u)] ^
	       T[7 * 256 + (la & 255u)];
}

// lport = htons(port): data bytes 10, 11 = port >> 8, port & 255.
__device__ __forceinline__ uint32_t hash_lp(const uint32_t *T, uint32_t lp)
{
	return T[10 * 256 + (lp >> 8)] ^ T[11 * 256 + (lp & 255u)];
}

template <bool FILTER>
__device__ __forceinline__ void cursor_at(Cursor &c, uint32_t idx, const DstParams &p, const uint32_t *T)
{
	const uint32_t q = idx / p.nf;
	c.fa = idx - q * p.nf;
	c.lp = q % kNEph;
	c.la = q / kNEph;
	if (FILTER)
		c.hl = hash_la(T, p.laddr_min + c.la) ^ p.hconst;
}

// idx += 64: at most one carry per digit (64 % nf < nf; 64 / nf + 1 < kNEph).
template <bool FILTER>
__device__ __forceinline__ void cursor_step64(Cursor &c, const DstParams &p, const uint32_t *T)
{
	c.fa += p.r64;
	const bool cf = c.fa >= p.nf;
	c.fa -= cf ? p.nf : 0u;
	c.lp += p.q64 + (cf ? 1u : 0u);
	if (c.lp >= kNEph) {
		c.lp -= kNEph;
		c.la++;
		if (FILTER)
			c.hl = hash_la(T, p.laddr_min + c.la) ^ p.hconst;
	}
}

// Does the tuple under the cursor pass the RSS filter (con-gen.c:337-342)?
__device__ __forceinline__ bool rss_pass(const Cursor &c, const DstParams &p, const uint32_t *T)
{
	const uint32_t h = (hash_fa(T, p.faddr_min + c.fa) ^ hash_lp(T, kEphMin + c.lp) ^ c.hl) & 0x7Fu;
	const uint32_t w = h < 64 ? (uint32_t)(p.pass_lo >> (h & 32)) : (uint32_t)(p.pass_hi >> (h & 32));
	return (w >> (h & 31)) & 1u;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
#pragma unroll
	for (int o = 32; o > 0; o >>= 1)
		v += __shfl_xor(v, o, 64);
	return v;
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t m)
{
	return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Exclusive prefix of tile t: the sum of the published counts of the tiles
// before it, walking back from t-1 until an inclusive word.  Each round
// trip reads 64 x kLookWin words (lane l, slot k: tile t-1-l-64k), so the
// walk crosses the tiles in flight in a few round trips.  Wave-uniform.
__device__ uint32_t dst_lookback(const DstParams &p, uint32_t t, int lane)
{
	uint64_t CGCK_GLOBAL *st = (uint64_t CGCK_GLOBAL *)p.status;
	uint32_t excl = 0;
	int64_t j = (int64_t)t - 1;
	uint32_t spins = 0;
	for (;;) {
		uint64_t s[kLookWin];
#pragma unroll
		for (int k = 0; k < kLookWin; k++) {
			const int64_t idx = j - lane - 64 * k;
			s[k] = idx >= 0 ? __hip_atomic_load(st + idx, RLX_AGENT) : kStIncl;
		}
		// nearest inclusive word: slot k, lane ctz
		int stop_k = kLookWin, stop_l = 63;
		bool missing = false;
#pragma unroll
		for (int k = 0; k < kLookWin; k++) {
			if (stop_k < kLookWin)
				break;
			const uint64_t incl = __ballot((s[k] >> 62) == 2);
			const uint64_t inval = __ballot((s[k] >> 62) == 0);
			const int l = incl ? __builtin_ctzll(incl) : 63;
			const uint64_t need = l >= 63 ? ~0ull : ((2ull << l) - 1);
			if (inval & need) {
				missing = true;
				break;
			}
			if (incl) {
				stop_k = k;
				stop_l = l;
			}
		}
		if (missing) {
			if (++spins > kSpinLimit) {
				if (lane == 0)
					__hip_atomic_store((uint32_t CGCK_GLOBAL *)p.ctl + 2, 1u, RLX_AGENT);
				return 0;
			}
			__builtin_amdgcn_s_sleep(1);
			continue;
		}
		uint32_t v = 0;
#pragma unroll
		for (int k = 0; k < kLookWin; k++)
			if (k < stop_k || (k == stop_k && lane <= stop_l))
				v += (uint32_t)s[k];
		excl += wave_sum(v);
		if (stop_k < kLookWin)
			return excl;
		j -= 64 * kLookWin;
	}
}

template <bool FILTER>
__global__ __launch_bounds__(256) void dst_cache_kernel(DstParams p)
{
	extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
	uint32_t *T = smem;                                                    // 12 x 256 (FILTER)
	uint32_t *B = smem + (FILTER ? 12 * 256 : 0);                          // [wave][iters/32][lane] bits
	uint32_t *S = B + kDstWaves * (kDstIters / 32) * 64;                   // [0] tile, [1..4] counts, [5] prefix
	uint32_t CGCK_GLOBAL *ctl = (uint32_t CGCK_GLOBAL *)p.ctl;
	uint64_t CGCK_GLOBAL *status = (uint64_t CGCK_GLOBAL *)p.status;
	u32x4_t CGCK_GLOBAL *out = (u32x4_t CGCK_GLOBAL *)p.out;
	const int lane = threadIdx.x & 63;
	const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	uint32_t *Bw = B + wave * (kDstIters / 32) * 64;
	if (FILTER) {
		const uint32_t CGCK_GLOBAL *gt = (const uint32_t CGCK_GLOBAL *)p.tab;
		for (uint32_t i = threadIdx.x; i < 12 * 256; i += 256)
			T[i] = gt[i];
	}
	for (;;) {
		if (threadIdx.x == 0) {
			uint32_t t = p.ntiles;
			if (!__hip_atomic_load(ctl + 1, RLX_AGENT))
				t = __hip_atomic_fetch_add(ctl + 0, 1u, RLX_AGENT);
			S[0] = t < p.ntiles ? t : p.ntiles;
		}
		__syncthreads();
		const uint32_t t = __builtin_amdgcn_readfirstlane(S[0]);
		if (t >= p.ntiles)
			break;
		const uint64_t base = (uint64_t)t * (kDstWaves * 64 * p.iters) + (uint64_t)wave * (64 * p.iters);
		const uint32_t start = (uint32_t)(base + lane < p.n ? base + lane : 0);

		// Pass 1: which tuples survive.  Lane bit u of word B[j0/32] = tuple
		// j*64 + lane of this wave; one LDS word per lane per 32 iterations.
		Cursor c;
		cursor_at<FILTER>(c, start, p, T);
		uint32_t cnt = 0;
		// tuples of this wave still below n, from this lane's first one
		const uint64_t left = base < p.n ? p.n - base : 0;
		const uint32_t rem = left > 0xffffffffu ? 0xffffffffu : (uint32_t)left;
		for (uint32_t j0 = 0; j0 < p.iters; j0 += 32) { // iters is a multiple of 32
			uint32_t bits = 0;
#pragma unroll 8
			for (uint32_t u = 0; u < 32; u++) {
				const bool in = (j0 + u) * 64 + lane < rem;
				const bool ok = FILTER ? in & rss_pass(c, p, T) : in;
				bits |= (ok ? 1u : 0u) << u;
				cursor_step64<FILTER>(c, p, T);
			}
			Bw[(j0 / 32) * 64 + lane] = bits;
			cnt += __builtin_popcount(bits);
		}
		cnt = wave_sum(cnt);
		if (lane == 0)
			S[1 + wave] = cnt;
		__syncthreads();
		const uint32_t A = S[1] + S[2] + S[3] + S[4];
		uint32_t wexcl = 0;
		for (int w = 0; w < wave; w++)
			wexcl += S[1 + w];

		// Publish, look back, publish the inclusive prefix.
		if (wave == 0) {
			uint32_t E = 0;
			if (t == 0) {
				if (lane == 0)
					__hip_atomic_store(status + 0, kStIncl | A, RLX_AGENT);
			} else {
				if (lane == 0)
					__hip_atomic_store(status + t, kStAgg | A, RLX_AGENT);
				E = dst_lookback(p, t, lane);
				if (lane == 0)
					__hip_atomic_store(status + t, kStIncl | (uint64_t)(E + A), RLX_AGENT);
			}
			if (lane == 0) {
				const uint32_t incl = E + A;
				if ((E < p.cap && incl >= p.cap) || t == p.ntiles - 1)
					*(uint32_t CGCK_GLOBAL *)p.count = incl < p.cap ? incl : p.cap;
				if (incl >= p.cap)
					__hip_atomic_store(ctl + 1, 1u, RLX_AGENT);
				S[5] = E;
			}
		}
		__syncthreads();
		const uint32_t E = __builtin_amdgcn_readfirstlane(S[5]);

		// Pass 2: write this tile's survivors at E + their rank, below cap.
		if (E < p.cap && cnt) {
			cursor_at<false>(c, start, p, T);
			uint32_t pos = E + wexcl;
			for (uint32_t j0 = 0; j0 < p.iters && pos < p.cap; j0 += 32) {
				const uint32_t bits = Bw[(j0 / 32) * 64 + lane];
				for (uint32_t u = 0; u < 32; u++) {
					const bool ok = (bits >> u) & 1u;
					const uint64_t m = __ballot(ok);
					const uint32_t at = pos + lanes_below(m);
					if (ok && at < p.cap) {
						const uint32_t fa = p.faddr_min + c.fa, la = p.laddr_min + c.la;
						const uint32_t lpb = __builtin_bswap16((uint16_t)(kEphMin + c.lp));
						const uint32_t fab = __builtin_bswap32(fa);
						// SO_HASH(faddr, lport, fport), subr.h:179-180
						const uint32_t soh = fab ^ (fab >> 16) ^ __builtin_bswap16((uint16_t)(lpb ^ p.fport_be));
						const u32x4_t e = {__builtin_bswap32(la), fab, lpb | (p.fport_be << 16), soh};
						out[at] = e;
					}
					pos += __builtin_popcountll(m);
					cursor_step64<false>(c, p, T);
				}
			}
		}
		__syncthreads(); // S and M are rewritten by the next tile
	}
}

// Expected tuples scanned before `cap` survivors exist: cap / (fraction of
// the 128 hash values that pass), or all of them.
static uint64_t dst_expected(uint32_t n, uint32_t cap, bool filter, uint64_t pass_lo, uint64_t pass_hi)
{
	const uint64_t pass = filter ? __builtin_popcountll(pass_lo) + __builtin_popcountll(pass_hi) : 128;
	const uint64_t want = pass ? (uint64_t)cap * 128 / pass + cap / 4 : n;
	return want < n ? want : n;
}

// Tile = 256 x iters tuples: 64 iterations per wave for long enumerations
// (the look-back is amortised over 16384 tuples), fewer for short ones so
// that they still spread over the chip (the reference's default, one laddr
// and one faddr, is 60536 tuples).
uint32_t dst_iters(uint32_t n, uint32_t cap, bool filter, uint64_t pass_lo, uint64_t pass_hi, int num_cus)
{
	const uint64_t work = dst_expected(n, cap, filter, pass_lo, pass_hi);
	const uint64_t per = work / ((uint64_t)num_cus * 256);
	if (const char *e = CGCK_ENV("CGCK_DST_ITERS")) // A/B sweeps (tools/rss_bench.py)
		return (uint32_t)atoi(e);
	uint32_t it = 32;
	while (it < (uint32_t)kDstIters && it < per)
		it *= 2;
	return it;
}

// Grid: enough workgroups for the expected work (a workgroup in flight
// finishes the tile it drew), at most 4 per CU.
hipError_t launch_dst_cache(const DstParams &p, int num_cus, hipStream_t st)
{
	if (p.ntiles == 0)
		return hipSuccess;
	const uint64_t tile = (uint64_t)kDstWaves * 64 * p.iters;
	uint64_t g = (dst_expected(p.n, p.cap, p.filter, p.pass_lo, p.pass_hi) + 2 * tile - 1) / tile;
	uint64_t gmax = (uint64_t)num_cus * 4;
	if (const char *e = CGCK_ENV("CGCK_DST_WGS")) // A/B sweeps: workgroups per CU
		gmax = (uint64_t)num_cus * atoi(e);
	g = g < 8 ? 8 : g;
	g = g > gmax ? gmax : g;
	g = g > p.ntiles ? p.ntiles : g;
	const size_t lds = (p.filter ? 12 * 256 * 4 : 0) + kDstMaskBytes + 64;
	if (p.filter) {
		CGCK_NOTE_KERNEL("dst_cache_kernel<true>");
		hipLaunchKernelGGL(dst_cache_kernel<true>, dim3((unsigned)g), dim3(256), lds, st, p);
	} else {
		CGCK_NOTE_KERNEL("dst_cache_kernel<false>");
		hipLaunchKernelGGL(dst_cache_kernel<false>, dim3((unsigned)g), dim3(256), lds, st, p);
	}
	return hipGetLastError();
}

} // namespace cgck
