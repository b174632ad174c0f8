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

hipError_t launch_toeplitz(const RssParams &p, int num_cus, hipStream_t st)
{
	if (p.n == 0)
		return hipSuccess;
	const uint64_t want = (p.n + 255) / 256;
	const uint64_t cap = (uint64_t)num_cus * 8;
	const dim3 g((unsigned)(want < cap ? want : cap)), b(256);
	const bool aligned = ((uintptr_t)p.data & 3) == 0 && (p.stride & 3) == 0;
	const bool lds = p.cnt <= kRssLdsMaxCnt;
	const size_t sh = lds ? (size_t)p.cnt * 256 * 4 : 0;
	if (aligned && p.cnt == 12)
		hipLaunchKernelGGL((toeplitz_kernel<3, true>), g, b, sh, st, p);
	else if (aligned && p.cnt == 36)
		hipLaunchKernelGGL((toeplitz_kernel<9, true>), g, b, sh, st, p);
	else if (lds)
		hipLaunchKernelGGL((toeplitz_kernel<0, true>), g, b, sh, st, p);
	else
		hipLaunchKernelGGL((toeplitz_kernel<0, false>), g, b, 0, st, p);
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

constexpr int kDstWaves = 4, kDstIters = 16;
constexpr uint32_t kNEph = 65535 - 5000 + 1; // NEPHEMERAL (subr.h:62-64)
constexpr uint32_t kEphMin = 5000;           // EPHEMERAL_MIN
constexpr uint64_t kStAgg = 1ull << 62, kStIncl = 2ull << 62;
constexpr uint32_t kSpinLimit = 1u << 22;

struct Cursor {
	uint32_t fa, lp, la; // offsets into the faddr, lport and laddr ranges
};

__device__ __forceinline__ void cursor_at(Cursor &c, uint32_t idx, const DstParams &p)
{
	const uint32_t q = idx / p.nf;
	c.fa = idx - q * p.nf;
	c.lp = q % kNEph;
	c.la = q / kNEph;
}

// idx += 64: at most one carry per digit (64 % nf < nf; 64 / nf + 1 < kNEph).
__device__ __forceinline__ void cursor_step64(Cursor &c, const DstParams &p)
{
	c.fa += p.r64;
	uint32_t dq = p.q64;
	if (c.fa >= p.nf) {
		c.fa -= p.nf;
		dq++;
	}
	c.lp += dq;
	if (c.lp >= kNEph) {
		c.lp -= kNEph;
		c.la++;
	}
}

// rss_hash4 data bytes (subr.c:513-521): faddr, laddr (network order =
// host-order value MSB first), fport as stored, lport = htons(port).  The
// fport bytes are constant per launch and folded into p.hconst.
__device__ __forceinline__ uint32_t tuple_hash(const uint32_t *T, uint32_t fa, uint32_t la, uint32_t lp,
					       uint32_t hconst)
{
	uint32_t h = hconst;
	h ^= T[0 * 256 + (fa >> 24)] ^ T[1 * 256 + ((fa >> 16) & 255u)];
	h ^= T[2 * 256 + ((fa >> 8) & 255u)] ^ T[3 * 256 + (fa & 255u)];
	h ^= T[4 * 256 + (la >> 24)] ^ T[5 * 256 + ((la >> 16) & 255u)];
	h ^= T[6 * 256 + ((la >> 8) & 255u)] ^ T[7 * 256 + (la & 255u)];
	h ^= T[10 * 256 + (lp >> 8)] ^ T[11 * 256 + (lp & 255u)];
	return h;
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

// Exclusive prefix of tile t: sum of the published counts of tiles < t,
// walking back from t-1 until an inclusive word.  Wave-uniform result.
__device__ uint32_t dst_lookback(const DstParams &p, uint32_t t, int lane)
{
	uint64_t CGCK_GLOBAL *st = (uint64_t CGCK_GLOBAL *)p.status;
	uint32_t excl = 0;
	int64_t j = (int64_t)t - 1;
	uint32_t spins = 0;
	for (;;) {
		const int64_t idx = j - lane;
		const uint64_t s = idx >= 0 ? __hip_atomic_load(st + idx, RLX_AGENT) : kStIncl;
		const uint64_t incl = __ballot((s >> 62) == 2);
		const uint64_t inval = __ballot((s >> 62) == 0);
		const int stop = incl ? __builtin_ctzll(incl) : 64;
		const uint64_t need = stop >= 63 ? ~0ull : ((2ull << stop) - 1);
		if (inval & need) {
			if (++spins > kSpinLimit) {
				if (lane == 0)
					__hip_atomic_store((uint32_t CGCK_GLOBAL *)p.ctl + 2, 1u, RLX_AGENT);
				return 0;
			}
			__builtin_amdgcn_s_sleep(1);
			continue;
		}
		excl += wave_sum(lane <= stop ? (uint32_t)s : 0u);
		if (stop < 64)
			return excl;
		j -= 64;
	}
}

template <bool FILTER>
__global__ __launch_bounds__(256) void dst_cache_kernel(DstParams p)
{
	extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
	uint32_t *T = smem;                            // 12 x 256 tables (FILTER)
	uint32_t *S = smem + (FILTER ? 12 * 256 : 0);  // [0] tile, [1..4] wave counts, [5] tile prefix
	uint32_t CGCK_GLOBAL *ctl = (uint32_t CGCK_GLOBAL *)p.ctl;
	uint64_t CGCK_GLOBAL *status = (uint64_t CGCK_GLOBAL *)p.status;
	u32x4_t CGCK_GLOBAL *out = (u32x4_t CGCK_GLOBAL *)p.out;
	const int lane = threadIdx.x & 63;
	const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
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
		const uint64_t base = (uint64_t)t * (kDstWaves * kDstIters * 64) + (uint64_t)wave * (kDstIters * 64);

		// Pass 1: which tuples survive (one ballot per 64).
		Cursor c;
		cursor_at(c, (uint32_t)(base + lane < p.n ? base + lane : 0), p);
		uint64_t m[kDstIters];
		uint32_t cnt = 0;
#pragma unroll
		for (int j = 0; j < kDstIters; j++) {
			bool ok = base + (uint64_t)(j * 64 + lane) < p.n;
			if (FILTER && ok) {
				const uint32_t h = tuple_hash(T, p.faddr_min + c.fa, p.laddr_min + c.la, kEphMin + c.lp,
							      p.hconst) & 0x7Fu;
				ok = ((h < 64 ? p.pass_lo >> h : p.pass_hi >> (h - 64)) & 1u) != 0;
			}
			m[j] = __ballot(ok);
			cnt += __builtin_popcountll(m[j]);
			cursor_step64(c, p);
		}
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
		if (E < p.cap) {
			cursor_at(c, (uint32_t)(base + lane < p.n ? base + lane : 0), p);
			uint32_t pos = E + wexcl;
#pragma unroll
			for (int j = 0; j < kDstIters; j++) {
				const uint32_t at = pos + lanes_below(m[j]);
				if (((m[j] >> lane) & 1u) && at < p.cap) {
					const uint32_t fa = p.faddr_min + c.fa, la = p.laddr_min + c.la;
					const uint32_t lpb = __builtin_bswap16((uint16_t)(kEphMin + c.lp));
					const uint32_t fab = __builtin_bswap32(fa);
					// SO_HASH(faddr, lport, fport), subr.h:179-180
					const uint32_t soh = fab ^ (fab >> 16) ^ __builtin_bswap16((uint16_t)(lpb ^ p.fport_be));
					const u32x4_t e = {__builtin_bswap32(la), fab, lpb | (p.fport_be << 16), soh};
					out[at] = e;
				}
				pos += __builtin_popcountll(m[j]);
				cursor_step64(c, p);
			}
		}
		__syncthreads(); // S is rewritten by the next tile
	}
}

hipError_t launch_dst_cache(const DstParams &p, int num_cus, hipStream_t st)
{
	if (p.ntiles == 0)
		return hipSuccess;
	const uint32_t cap = (uint32_t)num_cus * 8;
	const dim3 g(p.ntiles < cap ? p.ntiles : cap), b(256);
	if (p.filter)
		hipLaunchKernelGGL(dst_cache_kernel<true>, g, b, (12 * 256 + 16) * 4, st, p);
	else
		hipLaunchKernelGGL(dst_cache_kernel<false>, g, b, 16 * 4, st, p);
	return hipGetLastError();
}

} // namespace cgck
