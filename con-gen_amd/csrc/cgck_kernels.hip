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

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// Streaming chunk load; NT = nontemporal (read-once data, no cache retention).
template <bool NT>
__device__ __forceinline__ uint4 ld(const uint4 *p)
{
	if (NT) {
		u32x4_t x = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t *>(p));
		return make_uint4(x[0], x[1], x[2], x[3]);
	}
	return *p;
}

template <bool NT>
struct GChunks {
	const uint4 *p;
	__device__ __forceinline__ uint4 operator[](int i) const { return ld<NT>(p + i); }
};

// Block-iteration schedule: contiguous ranges per block (p.contig) or
// grid-stride.  Contiguous ranges keep each block's stream sequential in HBM.
struct Sched {
	uint64_t it, end, step;
};

__device__ __forceinline__ Sched sched(uint64_t n_iters, bool contig)
{
	Sched s;
	if (contig) {
		const uint64_t per = (n_iters + gridDim.x - 1) / gridDim.x;
		s.it = (uint64_t)blockIdx.x * per;
		s.end = s.it + per < n_iters ? s.it + per : n_iters;
		s.step = 1;
	} else {
		s.it = blockIdx.x;
		s.end = n_iters;
		s.step = gridDim.x;
	}
	return s;
}

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

template <int G, int S, int U, bool DESC, bool NT>
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

	const Sched sc = sched((p.n + PPB - 1) / PPB, p.contig);
	for (uint64_t blk = sc.it; blk < sc.end; blk += sc.step) {
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
				v[u][s] = k < nch[u] ? ld<NT>(c0 + k) : make_uint4(0, 0, 0, 0);
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
				uint4 w = k < nch[u] ? ld<NT>(c0 + k) : make_uint4(0, 0, 0, 0);
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
// Lane-per-packet kernel (small and mixed-size packets)
//
// One lane owns one packet, so nothing crosses lanes: the lane streams its
// packet's 16-byte chunks 8 at a time (one 128-byte line per lane per step)
// and sums them RAW (4 v_dot2 per chunk, no masks).  Per-packet work runs
// once per lane, i.e. once per packet, not once per lane of a group:
//   * tot = raw sum - bytes of chunk 0 before the packet - bytes of the last
//     chunk after it (two masked sums, skipped wave-uniformly when aligned);
//   * the header zone [ip, ip+80) is realigned into 20 packet-relative
//     dwords (v_alignbyte over a 4-way select), after which the IP sum,
//     pseudo src/dst, protocol and both checksum fields sit at fixed or
//     hl-indexed dword positions;
//   * zeroed-field semantics are applied by one's-complement subtraction of
//     the field values from the sums that cover them.
// --------------------------------------------------------------------------

// (m & a) | (~m & b): one v_bfi_b32.  The mask is made opaque to the
// optimizer so selects between array elements are never rewritten into a
// dynamically indexed (scratch) load.
__device__ __forceinline__ uint32_t pick(uint32_t m, uint32_t a, uint32_t b)
{
	return (a & m) | (b & ~m);
}

__device__ __forceinline__ uint32_t opaque(uint32_t m)
{
	asm volatile("" : "+v"(m));
	return m;
}

// x - y in one's-complement (mod 65535) on folded 16-bit values.
__device__ __forceinline__ uint32_t ocsub(uint32_t x, uint32_t y)
{
	return fold16(x + (0xffffu - y));
}

// One packet on one lane.  v[0..S0) hold chunks 0..S0-1 (zero past nch),
// `last` the packet's last chunk.
template <int S0, class Chunks>
__device__ __forceinline__ void lpp_packet(const KParams &p, uint64_t k, bool ok, uint64_t a0, int len,
					   const uint4 (&v)[S0], const uint4 &last, Chunks c0)
{
	static_assert(S0 >= 6, "the header zone spans chunks 0..5");
	const uint32_t flags = p.flags;
	const bool raw = flags & CGCK_RAW;
	const int q = (int)(a0 & 15);
	const int nch = len ? (int)(((a0 + len + 15) >> 4) - (a0 >> 4)) : 0;

	uint32_t tot = 0;
#pragma unroll
	for (int i = 0; i < S0; ++i)
		if (__any(i < nch))
			tot = sum4(v[i], tot);

	// Header zone, packet-relative dwords (while the rest streams in).
	uint32_t hd = 0, ip = 0, ps = 0, proto = 0, fip = 0, fl4 = 0;
	int fo = -1;
	if (!raw) {
		uint32_t D[24];
#pragma unroll
		for (int i = 0; i < 6; ++i) {
			D[4 * i + 0] = v[i].x;
			D[4 * i + 1] = v[i].y;
			D[4 * i + 2] = v[i].z;
			D[4 * i + 3] = v[i].w;
		}
		const int qd = q >> 2, qb = q & 3;
		const bool unaligned = __any(qb != 0);
		const bool shifted = __any(qd != 0);
		// S[i] = dword qd + i of the chunk run (two select stages), then
		// R[i] = bytes [q + 4i, q + 4i + 4) via v_alignbyte.
		uint32_t S[21];
		if (shifted) {
			const uint32_t m1 = opaque((qd & 1) ? ~0u : 0u);
			const uint32_t m2 = opaque((qd & 2) ? ~0u : 0u);
			uint32_t E[23];
#pragma unroll
			for (int i = 0; i < 23; ++i)
				E[i] = pick(m1, D[i + 1], D[i]);
#pragma unroll
			for (int i = 0; i < 21; ++i)
				S[i] = pick(m2, E[i + 2], E[i]);
		} else {
#pragma unroll
			for (int i = 0; i < 21; ++i)
				S[i] = D[i];
		}
		uint32_t R[20];
#pragma unroll
		for (int i = 0; i < 20; ++i)
			R[i] = unaligned ? __builtin_amdgcn_alignbyte(S[i + 1], S[i], (uint32_t)qb) : S[i];
		hd = R[0] & 15;
		proto = (R[2] >> 8) & 0xffu;
		fip = R[2] >> 16;
		// wave-uniform bound on the dwords any lane needs (OR >= max)
		uint32_t hor = 0;
#pragma unroll
		for (int b = 0; b < 4; ++b)
			hor |= __any((hd >> b) & 1) ? (1u << b) : 0u;
		const bool need_f = (flags & (CGCK_VERIFY | CGCK_ZERO_FIELDS | CGCK_STORE)) && (flags & CGCK_L4);
		const int nmax = (int)hor + (need_f ? 5 : 0);
		const int hl = (int)hd * 4;
		if (need_f && len >= 20 && len >= hl) {
			const int f = l4_field(proto, flags);
			if (f >= 0 && hl + f + 2 <= len)
				fo = f;
		}
		const int fi = fo >= 0 ? (hl + fo) >> 2 : -1;
		uint32_t fw = 0;
#pragma unroll
		for (int i = 0; i < 20; ++i) {
			if (i < (int)hor || i < 5)
				ip = hsum((uint32_t)i < hd ? R[i] : 0u, ip);
			if (need_f && i < nmax)
				fw = i == fi ? R[i] : fw;
		}
		fl4 = (fo & 2) ? (fw >> 16) : (fw & 0xffffu);
		ps = hsum(R[4], hsum(R[3], 0));
	}

	// Remaining chunks except the last (held in `last`): raw sums only, 8
	// (one 128-byte line) per step.  Every byte is read exactly once: a STORE
	// batch may rewrite a neighbour's header inside our last chunk, so a
	// second read of it could differ from the first.
	const int nmid = nch - 1;
	for (int t = S0; __any(t < nmid); t += 8) {
		uint4 w[8];
#pragma unroll
		for (int i = 0; i < 8; ++i) {
			const int c = t + i;
			w[i] = c < nmid ? c0[c] : make_uint4(0, 0, 0, 0);
		}
		uint32_t s = 0;
#pragma unroll
		for (int i = 0; i < 8; ++i)
			s = sum4(w[i], s);
		tot = fold16(tot) + fold16(s);
	}

	// Exclude the bytes of the first/last chunk outside [q, q + len).
	if (__any(q != 0))
		tot = fold16(tot) + (0xffffu - fold16(msum(v[0], 0, 0, q, 0)));
	const int e = q + len - 16 * (nch - 1); // bytes of the last chunk inside
	if (__any(nch > S0)) {
		// last chunk not in v[]: add its in-packet bytes
		const uint32_t in_last = nch > S0 ? msum(last, 0, 0, e, 0) : 0u;
		tot = fold16(tot) + fold16(in_last);
	}
	if (__any(nch > 0 && nch <= S0 && e != 16))
		tot = fold16(tot) + (0xffffu - fold16(nch > 0 && nch <= S0 ? msum(last, 0, e, 16, 0) : 0u));
	uint32_t T = fold16(tot);
	if (q & 1)
		T = bswap16(T); // now packet-relative

	if (!ok)
		return;
	uint32_t lo = 0, hi = 0, verdict = 0;
	const int hl = (int)hd * 4;
	if (raw) {
		lo = finish(T);
	} else if (len < 20 || len < hl) {
		verdict = CGCK_BAD_LEN;
	} else {
		uint32_t IPs = fold16(ip), PS = fold16(ps);
		if (flags & (CGCK_ZERO_FIELDS | CGCK_VERIFY)) {
			T = ocsub(T, fip);
			if (hl >= 12)
				IPs = ocsub(IPs, fip);
			if (fo >= 0) {
				const int o = hl + fo;
				if (o != 10)
					T = ocsub(T, fl4);
				if (o >= 12 && o < 20)
					PS = ocsub(PS, fl4);
			}
		}
		if (flags & CGCK_IP)
			lo = finish(IPs);
		if (flags & CGCK_L4) {
			uint32_t L = ocsub(T, IPs);
			if (!(flags & CGCK_L4_NOPSEUDO))
				L = fold16(L + PS + (proto << 8) + bswap16((uint32_t)(len - hl) & 0xffffu));
			hi = finish(L);
		}
		if (flags & CGCK_VERIFY) {
			uint32_t want = fip;
			if ((flags & CGCK_V_IP_ZERO_IS_FFFF) && want == 0)
				want = 0xffffu;
			if ((flags & CGCK_IP) && lo != want)
				verdict |= CGCK_BAD_IP;
			if ((flags & CGCK_L4) && fo >= 0 &&
			    !((flags & CGCK_V_UDP_ZERO_SKIP) && proto == 17 && fl4 == 0) && hi != fl4)
				verdict |= CGCK_BAD_L4;
		}
		if (flags & CGCK_STORE) {
			uint8_t *ipp = reinterpret_cast<uint8_t *>(a0);
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

// U adjacent packets per lane (so a lane walks U * len contiguous bytes),
// S0 chunks per packet loaded up front.
template <bool DESC, int U, int S0, bool NT>
__global__ __launch_bounds__(256) void lpp_kernel(KParams p)
{
	const Sched sc = sched((p.n + 256 * U - 1) / (256 * U), p.contig);
	for (uint64_t it = sc.it; it < sc.end; it += sc.step) {
		const uint64_t base = it * 256 * U;
		Pkt pk[U];
		uint4 v[U][S0], last[U];
#pragma unroll
		for (int u = 0; u < U; ++u) {
			pk[u] = get_pkt<DESC>(p, base + (uint64_t)threadIdx.x * U + u);
			const uint64_t a0 = pk[u].a0;
			const int nch = pk[u].len ? (int)(((a0 + pk[u].len + 15) >> 4) - (a0 >> 4)) : 0;
			const uint4 *c0 = reinterpret_cast<const uint4 *>(a0 & ~(uint64_t)15);
#pragma unroll
			for (int i = 0; i < S0; ++i)
				v[u][i] = i < nch ? ld<NT>(c0 + i) : make_uint4(0, 0, 0, 0);
			last[u] = nch > S0 ? ld<NT>(c0 + nch - 1) : make_uint4(0, 0, 0, 0);
			if (nch > 0 && nch <= S0) {
				// last chunk already loaded: pick it without a dynamic index
#pragma unroll
				for (int i = 0; i < S0; ++i)
					if (i == nch - 1)
						last[u] = v[u][i];
			}
		}
#pragma unroll
		for (int u = 0; u < U; ++u)
			lpp_packet<S0>(p, base + (uint64_t)threadIdx.x * U + u, pk[u].ok, pk[u].a0,
				       (int)pk[u].len, v[u], last[u],
				       GChunks<NT>{reinterpret_cast<const uint4 *>(pk[u].a0 & ~(uint64_t)15)});
	}
}

// --------------------------------------------------------------------------
// Staged lane-per-packet kernel (dense small/mixed batches).
//
// Each wave owns a contiguous range of packet indices and walks it in
// sub-batches of up to 64 packets that are CONTIGUOUS in memory (packet l+1
// starts where packet l ends — dense strided batches, packed IMIX).  The
// sub-batch's byte span is DMA-loaded into the wave's LDS window with fully
// coalesced global_load_lds_dwordx4 (1 KiB per wave-instruction, no VGPRs),
// then every lane processes its packet from LDS exactly like lpp_kernel.
// Sub-batches that are not dense enough (gaps, ring slots) fall back to
// direct per-lane loads.
// --------------------------------------------------------------------------

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

template <bool DESC, int WCH>
__global__ __launch_bounds__(256) void lpps_kernel(KParams p)
{
	constexpr int S0 = 6;
	__shared__ uint4 lds[4][WCH];
	const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
	const uint64_t nwaves = (uint64_t)gridDim.x * 4;
	const uint64_t wid = (uint64_t)blockIdx.x * 4 + wv;
	const uint64_t per = (p.n + nwaves - 1) / nwaves;
	const uint64_t r0 = wid * per;
	const uint64_t r1 = r0 + per < p.n ? r0 + per : p.n;
	uint4 *win = &lds[wv][0];

	for (uint64_t cur = r0; cur < r1;) {
		const uint64_t k = cur + l;
		Pkt pk = get_pkt<DESC>(p, k < r1 ? k : p.n); // beyond the range: !ok
		const uint64_t a0 = pk.a0;
		const uint64_t span0 = __builtin_amdgcn_readfirstlane((uint32_t)a0) |
				       ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(a0 >> 32)) << 32);
		const uint64_t S = span0 & ~(uint64_t)15;
		const uint64_t end = a0 + pk.len;
		const uint32_t prev_lo = __shfl_up((uint32_t)end, 1, 64);
		const uint32_t prev_hi = __shfl_up((uint32_t)(end >> 32), 1, 64);
		const uint64_t prev_end = ((uint64_t)prev_hi << 32) | prev_lo;
		const bool bad = !pk.ok || ((end + 15 - S) >> 4) > (uint64_t)WCH || (l > 0 && a0 != prev_end);
		const uint64_t badm = __ballot(bad);
		const int m = badm ? __builtin_ctzll(badm) : 64;
		const int lim = (int)(r1 - cur < 64 ? r1 - cur : 64);
		if (m >= 48 || m == lim) {
			// Dense: stage [S, end of packet m-1) in LDS, coalesced.
			const uint32_t lastend_lo = __shfl((uint32_t)end, m - 1, 64);
			const uint32_t lastend_hi = __shfl((uint32_t)(end >> 32), m - 1, 64);
			const uint64_t lastend = ((uint64_t)lastend_hi << 32) | lastend_lo;
			const int C = (int)((lastend + 15 - S) >> 4);
			const uint4 *g = reinterpret_cast<const uint4 *>(S);
			for (int j0 = 0; j0 < C; j0 += 64) {
				if (j0 + l < C)
					__builtin_amdgcn_global_load_lds((glb_void_t *)(g + j0 + l),
									 (lds_void_t *)(win + j0), 16, 0, 0);
			}
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			if (l < m) {
				const int nch = pk.len ? (int)(((a0 + pk.len + 15) >> 4) - (a0 >> 4)) : 0;
				const uint4 *c0 = win + (((a0 & ~(uint64_t)15) - S) >> 4);
				uint4 v[S0];
#pragma unroll
				for (int i = 0; i < S0; ++i)
					v[i] = i < nch ? c0[i] : make_uint4(0, 0, 0, 0);
				uint4 last = nch > 0 ? c0[nch - 1] : make_uint4(0, 0, 0, 0);
				lpp_packet<S0>(p, k, true, a0, (int)pk.len, v, last, c0);
			}
			cur += m;
			// every lane's LDS reads are done before the next sub-batch's DMA
			// overwrites the window (reads complete in order within the wave)
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
		} else {
			// Sparse: direct per-lane loads for all `lim` packets.
			const int nch = pk.len ? (int)(((a0 + pk.len + 15) >> 4) - (a0 >> 4)) : 0;
			const uint4 *c0 = reinterpret_cast<const uint4 *>(a0 & ~(uint64_t)15);
			uint4 v[S0];
#pragma unroll
			for (int i = 0; i < S0; ++i)
				v[i] = i < nch ? c0[i] : make_uint4(0, 0, 0, 0);
			uint4 last = nch > S0 ? c0[nch - 1] : make_uint4(0, 0, 0, 0);
			if (nch > 0 && nch <= S0) {
#pragma unroll
				for (int i = 0; i < S0; ++i)
					if (i == nch - 1)
						last = v[i];
			}
			lpp_packet<S0>(p, k, pk.ok, a0, (int)pk.len, v, last, GChunks<false>{c0});
			cur += lim;
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

hipError_t launch_probe_read(const void *src, uint64_t bytes, uint32_t *sink, int num_cus, int variant,
			     hipStream_t st)
{
	const uint4 *s = reinterpret_cast<const uint4 *>(src);
	const uint64_t n = bytes / 16;
	switch (variant) {
	case 1:
		hipLaunchKernelGGL((probe_read_kernel<8, true>), dim3(num_cus * 8), dim3(256), 0, st, s, n, sink);
		break;
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
	default:
		hipLaunchKernelGGL((probe_read_kernel<8, false>), dim3(num_cus * 8), dim3(256), 0, st, s, n, sink);
	}
	return hipGetLastError();
}

// --------------------------------------------------------------------------
// Launchers
// --------------------------------------------------------------------------

template <int G, int S, int U, bool DESC>
static hipError_t launch_t(const KParams &p, int max_blocks, bool nt, hipStream_t st)
{
	constexpr uint64_t PPB = (256 / G) * U;
	uint64_t want = (p.n + PPB - 1) / PPB;
	int blocks = (int)(want < (uint64_t)max_blocks ? want : (uint64_t)max_blocks);
	if (blocks < 1)
		blocks = 1;
	if (nt)
		hipLaunchKernelGGL((cksum_kernel<G, S, U, DESC, true>), dim3(blocks), dim3(256), 0, st, p);
	else
		hipLaunchKernelGGL((cksum_kernel<G, S, U, DESC, false>), dim3(blocks), dim3(256), 0, st, p);
	return hipGetLastError();
}

template <bool DESC, int U, int S0>
static hipError_t launch_lpp(const KParams &p, int max_blocks, bool nt, hipStream_t st)
{
	uint64_t want = (p.n + 256 * U - 1) / (256 * U);
	int blocks = (int)(want < (uint64_t)max_blocks ? want : (uint64_t)max_blocks);
	if (blocks < 1)
		blocks = 1;
	if (nt)
		hipLaunchKernelGGL((lpp_kernel<DESC, U, S0, true>), dim3(blocks), dim3(256), 0, st, p);
	else
		hipLaunchKernelGGL((lpp_kernel<DESC, U, S0, false>), dim3(blocks), dim3(256), 0, st, p);
	return hipGetLastError();
}

template <bool DESC, int WCH>
static hipError_t launch_lpps(const KParams &p, int num_cus, hipStream_t st)
{
	// ~2 sub-batches of 64 packets per wave at least; at most 8 blocks per CU
	uint64_t want = (p.n + 4 * 128 - 1) / (4 * 128);
	uint64_t cap = (uint64_t)num_cus * 8;
	int blocks = (int)(want < cap ? want : cap);
	if (blocks < 1)
		blocks = 1;
	hipLaunchKernelGGL((lpps_kernel<DESC, WCH>), dim3(blocks), dim3(256), 0, st, p);
	return hipGetLastError();
}

// Family and shape selection.  `kernel` = variant | flags:
//   variant (bits 0-3): 0 auto, 1 group, 2 lane-per-packet (auto shape),
//     3 lpp U1/S8, 4 lpp U2/S6, 5 lpp U1/S6, 6 lpp U4/S6, 7 staged 4 KiB, 8 staged 24 KiB;
//   kNT (bit 4) nontemporal loads; kContig (bit 5) contiguous block ranges;
//   kExplicit (bit 6) use bits 4-5 as given instead of the defaults.
// max_len = the longest packet the batch may hold.
hipError_t launch_cksum(const KParams &p0, uint32_t max_len, int num_cus, int kernel, hipStream_t st)
{
	if (p0.n == 0)
		return hipSuccess;
	KParams p = p0;
	const bool d = p.desc != nullptr;
	const bool lpp_ok = !(p.flags & kFlagNoLenCheck);
	int variant = kernel & 15;
	if (variant == 0)
		variant = (lpp_ok && max_len < 1024) ? 2 : 1;
	if (variant >= 2 && !lpp_ok)
		variant = 1;
	if (variant == 2)
		variant = kDefaultLpp;
	bool nt, contig;
	if (kernel & kExplicit) {
		nt = kernel & kNT;
		contig = kernel & kContig;
	} else {
		nt = variant == 1 ? kDefaultGroupNT : kDefaultLppNT;
		contig = variant == 1 ? kDefaultGroupContig : kDefaultLppContig;
	}
	p.contig = contig;
	if (variant >= 3) {
		const int mb = num_cus * 8;
		switch (variant) {
		case 7:
			return d ? launch_lpps<true, 264>(p, num_cus, st) : launch_lpps<false, 264>(p, num_cus, st);
		case 8:
			return d ? launch_lpps<true, 1536>(p, num_cus, st) : launch_lpps<false, 1536>(p, num_cus, st);
		case 4:
			return d ? launch_lpp<true, 2, 6>(p, mb, nt, st) : launch_lpp<false, 2, 6>(p, mb, nt, st);
		case 5:
			return d ? launch_lpp<true, 1, 6>(p, mb, nt, st) : launch_lpp<false, 1, 6>(p, mb, nt, st);
		case 6:
			return d ? launch_lpp<true, 4, 6>(p, mb, nt, st) : launch_lpp<false, 4, 6>(p, mb, nt, st);
		default:
			return d ? launch_lpp<true, 1, 8>(p, mb, nt, st) : launch_lpp<false, 1, 8>(p, mb, nt, st);
		}
	}
	const int max_blocks = num_cus * 16;
	if (max_len <= 80) // <= 6 chunks at any alignment: two steps of 4 lanes
		return d ? launch_t<4, 2, 4, true>(p, max_blocks, nt, st)
			 : launch_t<4, 2, 4, false>(p, max_blocks, nt, st);
	if (max_len <= 256)
		return d ? launch_t<16, 2, 2, true>(p, max_blocks, nt, st)
			 : launch_t<16, 2, 2, false>(p, max_blocks, nt, st);
	if (max_len <= 1600)
		return d ? launch_t<16, 6, 1, true>(p, max_blocks, nt, st)
			 : launch_t<16, 6, 1, false>(p, max_blocks, nt, st);
	return d ? launch_t<64, 4, 1, true>(p, max_blocks, nt, st)
		 : launch_t<64, 4, 1, false>(p, max_blocks, nt, st);
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
