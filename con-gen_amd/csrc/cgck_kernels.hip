// cgck_kernels.hip — gfx950 (MI355X, CDNA4) kernels of the checksum engine.
//
// Replaces the arithmetic of con-gen's subr.c:119-223 (cksum_add, reduce,
// cksum_raw, in_cksum, pseudo_cksum, udp_cksum) for whole batches of packets.
//
// Arithmetic.  The reference sums native little-endian u64 words with an
// end-around carry and folds 64->32->16 (subr.c:127-184).  Because 2^16 == 1
// (mod 65535), any summation order and width gives the same residue, so the
// kernels sum 16-bit halves into u32 lane partials (one v_dot2_u32_u16 per
// dword: lo*1 + hi*1 + acc) and fold once per packet.  Words are counted in
// the ABSOLUTE address frame (16-byte aligned HBM chunks); for a packet that
// starts at an odd address the folded sum is byte-swapped (x256 mod 65535),
// which is exactly the reference's region-relative word pairing.  The
// complement and the 0 -> 0xFFFF rule of reduce() (subr.c:150-154) are applied
// last.
//
// Per packet three masked sums are formed from the same HBM stream:
//   tot = sum over [ip, ip+ip_len)           (all lanes)
//   ip  = sum over [ip, ip+ip_hl*4)          (header-zone lanes only)
//   ps  = sum over [ip+12, ip+20)            (src/dst of the pseudo-header)
// and the L4 sum is tot - ip (the two regions partition the datagram), plus
// ps, plus ip_p<<8 and htons(l4len) read as a little-endian word
// (struct pseudo, subr.c:119-125).
//
// Work mapping.  A group of G lanes (G = 4, 16 or 64) owns one packet at a
// time and walks its 16-byte chunks G at a time with coalesced uint4 loads,
// S steps unrolled so S loads per lane are in flight; U packets per group per
// iteration.  Group partials are reduced with DPP row operations (no LDS).
// No MFMA: this is a memory-bound integer reduction.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cgck_internal.h"

namespace cgck {

// --------------------------------------------------------------------------
// Lane helpers
// --------------------------------------------------------------------------

__device__ __forceinline__ uint32_t hsum(uint32_t w, uint32_t acc)
{
	// (w & 0xffff) + (w >> 16) + acc in one v_dot2_u32_u16.
	typedef unsigned short us2 __attribute__((ext_vector_type(2)));
	us2 a = __builtin_bit_cast(us2, w);
	us2 one = {1, 1};
	return __builtin_amdgcn_udot2(a, one, acc, false);
}

__device__ __forceinline__ uint32_t sum4(const uint4 &w, uint32_t acc)
{
	return hsum(w.w, hsum(w.z, hsum(w.y, hsum(w.x, acc))));
}

// Byte mask of bytes [s, e) of a dword, s, e already clamped to [0, 4].
__device__ __forceinline__ uint32_t bmask(int s, int e)
{
	uint32_t hm = e >= 4 ? 0xffffffffu : ((1u << (8 * e)) - 1u);
	uint32_t lm = 0xffffffffu << (8 * (s & 3));
	return e > s ? (hm & lm) : 0u;
}

__device__ __forceinline__ int clamp4(int x)
{
	return min(max(x, 0), 4);
}

// Mask of the bytes of dword i of the chunk at packet-relative byte co that
// fall inside [r0, r1) (packet-relative, relative to the 16-aligned c0).
__device__ __forceinline__ uint32_t dmask(int co, int i, int r0, int r1)
{
	int b = co + 4 * i;
	return bmask(clamp4(r0 - b), clamp4(r1 - b));
}

__device__ __forceinline__ uint32_t msum(const uint4 &w, int co, int r0, int r1, uint32_t acc)
{
	acc = hsum(w.x & dmask(co, 0, r0, r1), acc);
	acc = hsum(w.y & dmask(co, 1, r0, r1), acc);
	acc = hsum(w.z & dmask(co, 2, r0, r1), acc);
	acc = hsum(w.w & dmask(co, 3, r0, r1), acc);
	return acc;
}

__device__ __forceinline__ void zero_bytes(uint4 &w, int co, int r0, int r1)
{
	w.x &= ~dmask(co, 0, r0, r1);
	w.y &= ~dmask(co, 1, r0, r1);
	w.z &= ~dmask(co, 2, r0, r1);
	w.w &= ~dmask(co, 3, r0, r1);
}

// Group reduction over G lanes (G in {4, 8, 16, 32, 64}); every lane of the
// group ends with the group's sum.  quad_perm and row mirrors are DPP; the
// 32/64 steps use cross-row swizzles.
template <int G>
__device__ __forceinline__ uint32_t gsum(uint32_t v)
{
	// xor 1 and xor 2 inside quads
	v += __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false); // quad_perm [1,0,3,2]
	v += __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false); // quad_perm [2,3,0,1]
	if (G >= 8)
		v += __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, false); // row_half_mirror
	if (G >= 16)
		v += __builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, false); // row_mirror
	if (G >= 32)
		v += __shfl_xor(v, 16, 64);
	if (G >= 64)
		v += __shfl_xor(v, 32, 64);
	return v;
}

// Fold a u32 one's-complement partial to 16 bits (value in [0, 0xffff],
// congruent mod 65535).
__device__ __forceinline__ uint32_t fold16(uint32_t x)
{
	x = (x & 0xffffu) + (x >> 16);
	x = (x & 0xffffu) + (x >> 16);
	x = (x & 0xffffu) + (x >> 16);
	return x;
}

__device__ __forceinline__ uint32_t bswap16(uint32_t x)
{
	return ((x & 0xffu) << 8) | ((x >> 8) & 0xffu);
}

// reduce() of subr.c:137-156 applied to a folded, region-relative sum.
__device__ __forceinline__ uint32_t finish(uint32_t f)
{
	uint32_t r = (~f) & 0xffffu;
	return r ? r : 0xffffu;
}

__device__ __forceinline__ int l4_field(uint32_t proto, uint32_t flags)
{
	if (flags & CGCK_L4_NOPSEUDO)
		return proto == 1 ? 2 : -1;
	return proto == 6 ? 16 : (proto == 17 ? 6 : -1);
}

__device__ __forceinline__ void store16(uint8_t *p, uint32_t v)
{
	if ((reinterpret_cast<uintptr_t>(p) & 1) == 0) {
		*reinterpret_cast<uint16_t *>(p) = (uint16_t)v;
	} else {
		p[0] = (uint8_t)v;
		p[1] = (uint8_t)(v >> 8);
	}
}

// --------------------------------------------------------------------------
// The checksum kernel
// --------------------------------------------------------------------------

struct Pkt {
	uint64_t a0;  // absolute address of the IPv4 header (or region)
	uint32_t len; // bytes
	bool ok;      // packet index < n
};

template <bool DESC>
__device__ __forceinline__ Pkt get_pkt(const KParams &p, uint64_t k)
{
	Pkt r;
	r.ok = k < p.n;
	uint64_t kk = r.ok ? k : 0;
	if (DESC) {
		const uint32_t *d = reinterpret_cast<const uint32_t *>(p.desc) + 3 * kk;
		uint32_t lo = d[0], hi = d[1], w2 = d[2];
		uint64_t fo = ((uint64_t)hi << 32) | lo;
		r.a0 = reinterpret_cast<uint64_t>(p.base) + fo + (w2 & 0xffffu);
		r.len = w2 >> 16;
	} else {
		r.a0 = reinterpret_cast<uint64_t>(p.base) + kk * p.stride + p.l3_off;
		r.len = p.ip_len;
	}
	if (!r.ok)
		r.len = 0;
	return r;
}

// Per-packet, per-lane partial state.
struct Part {
	uint32_t tot, ip, ps, fld; // fld = stored ip field | stored l4 field << 16 (abs frame)
};

// Accumulate one loaded chunk (k = chunk index inside the packet).
template <bool HDR>
__device__ __forceinline__ void eat(Part &pt, uint4 w, int k, int q, int len, int hl, int fo,
				    uint32_t flags)
{
	const int co = k * 16;
	if (HDR && co < q + 80) {
		// Header zone: stored fields, optional zeroing, header sums.
		if (flags & (CGCK_VERIFY | CGCK_ZERO_FIELDS)) {
			uint32_t f = msum(w, co, q + 10, q + 12, 0);
			uint32_t g = fo >= 0 ? msum(w, co, q + hl + fo, q + hl + fo + 2, 0) : 0u;
			pt.fld += f | (g << 16);
			zero_bytes(w, co, q + 10, q + 12);
			if (fo >= 0)
				zero_bytes(w, co, q + hl + fo, q + hl + fo + 2);
		}
		pt.ip = msum(w, co, q, q + hl, pt.ip);
		pt.ps = msum(w, co, q + 12, q + 20, pt.ps);
	}
	if (co >= q && co + 16 <= q + len)
		pt.tot = sum4(w, pt.tot);
	else
		pt.tot = msum(w, co, q, q + len, pt.tot);
}

template <int G, int S, int U, bool DESC>
__global__ __launch_bounds__(256) void cksum_kernel(KParams p)
{
	constexpr int GPB = 256 / G;        // groups per block
	constexpr int PPB = GPB * U;        // packets per block iteration
	const int lane = threadIdx.x;
	const int gib = lane / G;           // group in block
	const int gl = lane % G;            // lane in group
	const uint32_t flags = p.flags;
	const bool raw = flags & CGCK_RAW;
	const bool need_hdr = !raw;

	for (uint64_t blk = blockIdx.x; blk * PPB < p.n; blk += gridDim.x) {
		Pkt pk[U];
		uint32_t b0[U], proto[U];
		uint4 v[U][S];
		int nch[U];
#pragma unroll
		for (int u = 0; u < U; ++u) {
			pk[u] = get_pkt<DESC>(p, blk * PPB + (uint64_t)u * GPB + gib);
			const uint64_t a0 = pk[u].a0;
			// Bytes read: the region, or (drop-in udp_cksum, host-guaranteed)
			// at least the 20 header bytes the pseudo-header needs.
			uint32_t span = pk[u].len;
			if ((flags & kFlagNoLenCheck) && pk[u].ok && span < 20)
				span = 20;
			nch[u] = span ? (int)(((a0 + span + 15) >> 4) - (a0 >> 4)) : 0;
			b0[u] = 0;
			proto[u] = 0;
			if (need_hdr && pk[u].ok && span > 0) {
				b0[u] = *reinterpret_cast<const uint8_t *>(a0);
				if (span > 9)
					proto[u] = *reinterpret_cast<const uint8_t *>(a0 + 9);
			}
			const uint4 *c0 = reinterpret_cast<const uint4 *>(a0 & ~(uint64_t)15);
#pragma unroll
			for (int s = 0; s < S; ++s) {
				const int k = s * G + gl;
				v[u][s] = k < nch[u] ? c0[k] : make_uint4(0, 0, 0, 0);
			}
		}
#pragma unroll
		for (int u = 0; u < U; ++u) {
			const int q = (int)(pk[u].a0 & 15);
			const int len = (int)pk[u].len;
			const int hl = (int)(b0[u] & 15) * 4;
			const int fo = (need_hdr && (flags & (CGCK_L4)) && len >= 20 && len >= hl &&
					l4_field(proto[u], flags) >= 0 &&
					hl + l4_field(proto[u], flags) + 2 <= len)
					       ? l4_field(proto[u], flags)
					       : -1;
			Part pt = {0, 0, 0, 0};
#pragma unroll
			for (int s = 0; s < S; ++s) {
				const int k = s * G + gl;
				if (need_hdr && s * G * 16 < 96)
					eat<true>(pt, v[u][s], k, q, len, hl, fo, flags);
				else
					eat<false>(pt, v[u][s], k, q, len, hl, fo, flags);
			}
			// Steps beyond the unrolled S (long packets): one at a time.
			const uint4 *c0 = reinterpret_cast<const uint4 *>(pk[u].a0 & ~(uint64_t)15);
			for (int s = S; __any(s * G < nch[u]); ++s) {
				const int k = s * G + gl;
				uint4 w = k < nch[u] ? c0[k] : make_uint4(0, 0, 0, 0);
				if (need_hdr && s * G * 16 < 96)
					eat<true>(pt, w, k, q, len, hl, fo, flags);
				else
					eat<false>(pt, w, k, q, len, hl, fo, flags);
				pt.tot = (pt.tot & 0xffffu) + (pt.tot >> 16); // keep u32 headroom
			}

			uint32_t tot = gsum<G>(pt.tot);
			uint32_t ip = 0, ps = 0, fld = 0;
			if (need_hdr) {
				ip = gsum<(G < 8 ? G : 8)>(pt.ip);
				ps = gsum<(G < 8 ? G : 8)>(pt.ps);
				fld = gsum<(G < 8 ? G : 8)>(pt.fld);
			}
			if (gl != 0 || !pk[u].ok)
				continue; // lane 0 of the group finishes the packet

			const uint64_t k = blk * PPB + (uint64_t)u * GPB + gib;
			const bool odd = q & 1;
			uint32_t lo = 0, hi = 0, verdict = 0;
			if (raw) {
				uint32_t f = fold16(tot);
				lo = finish(odd ? bswap16(f) : f);
			} else if (!(flags & kFlagNoLenCheck) && (len < 20 || len < hl)) {
				verdict = CGCK_BAD_LEN;
			} else {
				if (flags & CGCK_IP) {
					uint32_t f = fold16(ip);
					lo = finish(odd ? bswap16(f) : f);
				}
				if (flags & CGCK_L4) {
					const uint32_t l4len = (uint32_t)(len - hl);
					// L4 region = datagram minus header: one's-complement
					// subtraction, tot + ~ip (mod 65535).
					const uint32_t l4 = fold16(tot) + (0xffffu - fold16(ip));
					if (flags & CGCK_L4_NOPSEUDO) {
						uint32_t f = fold16(l4);
						hi = finish(odd ? bswap16(f) : f);
					} else {
						uint32_t f = fold16(l4 + ps);
						f = odd ? bswap16(f) : f;
						f += (proto[u] << 8) + bswap16(l4len & 0xffffu);
						hi = finish(fold16(f));
					}
				}
				if (flags & CGCK_VERIFY) {
					uint32_t sip = fld & 0xffffu, sl4 = fld >> 16;
					if (odd) {
						sip = bswap16(sip);
						sl4 = bswap16(sl4);
					}
					uint32_t want = sip;
					if ((flags & CGCK_V_IP_ZERO_IS_FFFF) && want == 0)
						want = 0xffffu;
					if ((flags & CGCK_IP) && lo != want)
						verdict |= CGCK_BAD_IP;
					if ((flags & CGCK_L4) && fo >= 0 &&
					    !((flags & CGCK_V_UDP_ZERO_SKIP) && proto[u] == 17 && sl4 == 0) &&
					    hi != sl4)
						verdict |= CGCK_BAD_L4;
				}
				if (flags & CGCK_STORE) {
					uint8_t *ipp = reinterpret_cast<uint8_t *>(pk[u].a0);
					if (flags & CGCK_IP)
						store16(ipp + 10, lo);
					if ((flags & CGCK_L4) && fo >= 0)
						store16(ipp + hl + fo, hi);
				}
			}
			if (p.out)
				p.out[k] = lo | (hi << 16);
			if (p.verdict)
				p.verdict[k] = (uint8_t)verdict;
			if (p.bad) {
				if (verdict & CGCK_BAD_IP)
					atomicAdd(p.bad + 0, 1u);
				if (verdict & CGCK_BAD_L4)
					atomicAdd(p.bad + 1, 1u);
			}
		}
	}
}

// --------------------------------------------------------------------------
// Synthetic input: byte j of the stream = byte j&7 of
// splitmix64(seed, j>>3); then per-packet header stamps.
// --------------------------------------------------------------------------

__device__ __forceinline__ uint64_t splitmix64(uint64_t seed, uint64_t j)
{
	uint64_t z = seed + (j + 1) * 0x9e3779b97f4a7c15ull;
	z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
	z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
	return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void synth_fill_kernel(uint8_t *base, uint64_t nbytes, uint64_t seed)
{
	const uint64_t nw = nbytes >> 3;
	uint64_t *w = reinterpret_cast<uint64_t *>(base);
	for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; 2 * i < nw;
	     i += (uint64_t)gridDim.x * 256) {
		uint64_t j = 2 * i;
		if (j + 1 < nw) {
			ulonglong2 x = make_ulonglong2(splitmix64(seed, j), splitmix64(seed, j + 1));
			*reinterpret_cast<ulonglong2 *>(w + j) = x;
		} else {
			w[j] = splitmix64(seed, j);
		}
	}
	if (blockIdx.x == 0 && threadIdx.x < (nbytes & 7)) {
		uint64_t b = (nw << 3) + threadIdx.x;
		base[b] = (uint8_t)(splitmix64(seed, b >> 3) >> (8 * (b & 7)));
	}
}

__device__ __forceinline__ void stamp(uint8_t *ip, uint32_t len)
{
	ip[0] = 0x45;
	ip[1] = 0;
	ip[2] = (uint8_t)(len >> 8);
	ip[3] = (uint8_t)len;
	ip[9] = 6;
	ip[10] = 0;
	ip[11] = 0;
	if (len >= 38) {
		ip[36] = 0;
		ip[37] = 0;
	}
}

__global__ __launch_bounds__(256) void synth_stamp_strided_kernel(uint8_t *base, uint64_t n,
								  uint64_t stride, uint32_t len)
{
	for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < n;
	     k += (uint64_t)gridDim.x * 256)
		stamp(base + k * stride, len);
}

__constant__ uint16_t c_imix_len[12] = {64, 576, 64, 64, 576, 64, 1500, 64, 576, 64, 64, 576};
__constant__ uint16_t c_imix_off[12] = {0, 64, 640, 704, 768, 1344, 1408, 2908, 2972, 3548, 3612, 3676};

__global__ __launch_bounds__(256) void synth_imix_kernel(uint8_t *base, uint32_t *desc, uint64_t n)
{
	for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < n;
	     k += (uint64_t)gridDim.x * 256) {
		uint64_t off = (k / 12) * (uint64_t)kImixCycleBytes + c_imix_off[k % 12];
		uint32_t len = c_imix_len[k % 12];
		stamp(base + off, len);
		desc[3 * k + 0] = (uint32_t)off;
		desc[3 * k + 1] = (uint32_t)(off >> 32);
		desc[3 * k + 2] = len << 16; // l3_off 0, ip_len
	}
}

// --------------------------------------------------------------------------
// Launchers
// --------------------------------------------------------------------------

template <int G, int S, int U, bool DESC>
static hipError_t launch_t(const KParams &p, int max_blocks, hipStream_t st)
{
	constexpr uint64_t PPB = (256 / G) * U;
	uint64_t want = (p.n + PPB - 1) / PPB;
	int blocks = (int)(want < (uint64_t)max_blocks ? want : (uint64_t)max_blocks);
	if (blocks < 1)
		blocks = 1;
	hipLaunchKernelGGL((cksum_kernel<G, S, U, DESC>), dim3(blocks), dim3(256), 0, st, p);
	return hipGetLastError();
}

// Shape selection: G lanes per packet and S unrolled steps from the packet
// length class (max_len = the longest packet the batch may hold).
hipError_t launch_cksum(const KParams &p, uint32_t max_len, int num_cus, hipStream_t st)
{
	if (p.n == 0)
		return hipSuccess;
	const int max_blocks = num_cus * 16;
	const bool d = p.desc != nullptr;
	if (max_len <= 80) // <= 6 chunks at any alignment: two steps of 4 lanes
		return d ? launch_t<4, 2, 4, true>(p, max_blocks, st)
			 : launch_t<4, 2, 4, false>(p, max_blocks, st);
	if (max_len <= 256)
		return d ? launch_t<16, 2, 2, true>(p, max_blocks, st)
			 : launch_t<16, 2, 2, false>(p, max_blocks, st);
	if (max_len <= 1600)
		return d ? launch_t<16, 6, 1, true>(p, max_blocks, st)
			 : launch_t<16, 6, 1, false>(p, max_blocks, st);
	return d ? launch_t<64, 4, 1, true>(p, max_blocks, st)
		 : launch_t<64, 4, 1, false>(p, max_blocks, st);
}

hipError_t launch_synth_fill(uint8_t *base, uint64_t nbytes, uint64_t seed, int num_cus, hipStream_t st)
{
	uint64_t want = (nbytes / 16 + 255) / 256;
	int blocks = (int)(want < (uint64_t)num_cus * 8 ? want : (uint64_t)num_cus * 8);
	if (blocks < 1)
		blocks = 1;
	hipLaunchKernelGGL(synth_fill_kernel, dim3(blocks), dim3(256), 0, st, base, nbytes, seed);
	return hipGetLastError();
}

hipError_t launch_synth_stamp(uint8_t *base, uint64_t n, uint64_t stride, uint32_t len, int num_cus,
			      hipStream_t st)
{
	uint64_t want = (n + 255) / 256;
	int blocks = (int)(want < (uint64_t)num_cus * 8 ? want : (uint64_t)num_cus * 8);
	if (blocks < 1)
		blocks = 1;
	hipLaunchKernelGGL(synth_stamp_strided_kernel, dim3(blocks), dim3(256), 0, st, base, n, stride, len);
	return hipGetLastError();
}

hipError_t launch_synth_imix(uint8_t *base, uint32_t *desc, uint64_t n, int num_cus, hipStream_t st)
{
	uint64_t want = (n + 255) / 256;
	int blocks = (int)(want < (uint64_t)num_cus * 8 ? want : (uint64_t)num_cus * 8);
	if (blocks < 1)
		blocks = 1;
	hipLaunchKernelGGL(synth_imix_kernel, dim3(blocks), dim3(256), 0, st, base, desc, n);
	return hipGetLastError();
}

} // namespace cgck
