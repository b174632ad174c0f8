// cgck_lane.hip — kernels whose per-packet work runs on ONE lane.
//
// The streaming rate of this path is VALU-issue-bound long before it is
// HBM-bound (tools/probe.py: ~300 extra VALU per 4 KiB halves a 64 B-packet
// stream), so per-packet work must run once per packet, not once per lane of
// a group, and must be cheap in the common cases.  Two kernels:
//
//  * lpp_kernel  — one lane per packet (small packets: every lane is a head).
//  * slot_kernel — one lane per 128-byte SLOT: a packet of L bytes spans
//    ceil(chunks/8) consecutive lanes of a wave, so mixed sizes (IMIX) keep
//    every lane loading 8 chunks at once, large packets load coalesced
//    across lanes, and the per-packet work (header, finish) runs on the
//    packet's head lane only.  Slot partial sums are joined by a segmented
//    suffix reduction towards the head lane.
//
// Shared per-packet pieces:
//  * header(): the first 6 chunks realigned to packet-relative dwords
//    (v_bfi selects + v_alignbyte) — IP header sum, pseudo src/dst, ip_p and
//    both stored checksum fields, with wave-uniform fast paths (all packets
//    16-byte aligned / dword aligned / ip_hl == 5);
//  * edges: the bytes of the first/last chunk outside the packet are taken
//    out of the raw chunk sum (each chunk is read exactly once — a STORE batch
//    may rewrite a neighbour's header inside our last chunk);
//  * finish(): zero-field semantics by one's-complement subtraction, the
//    pseudo-header, reduce() (subr.c:137-156), verdicts, stores, outputs.
#include "cgck_device.h"

namespace cgck {

// --------------------------------------------------------------------------
// Header zone
// --------------------------------------------------------------------------

struct Hdr {
	uint32_t hd;    // ip_hl (dwords)
	uint32_t ip;    // u32 partial over [0, 4*hd)
	uint32_t ps;    // u32 partial over [12, 20)
	uint32_t proto; // ip_p
	uint32_t fip;   // stored ip_sum as a host u16
	uint32_t fl4;   // stored L4 checksum (when fo >= 0)
	int fo;         // L4 field offset after the header, or -1
};

struct Align {
	int qb;
	bool shifted, unaligned;
	uint32_t m1, m2;
};

// dword qd + i of the chunk run (D = chunks 0..5), no dynamic register index
__device__ __forceinline__ uint32_t sdw(const uint32_t (&D)[24], int i, const Align &a)
{
	if (!a.shifted)
		return D[i];
	return pick(a.m2, pick(a.m1, D[i + 3], D[i + 2]), pick(a.m1, D[i + 1], D[i]));
}

// packet-relative dword i = bytes [q + 4i, q + 4i + 4)
__device__ __forceinline__ uint32_t rdw(const uint32_t (&D)[24], int i, const Align &a)
{
	const uint32_t lo = sdw(D, i, a);
	if (!a.unaligned)
		return lo;
	return __builtin_amdgcn_alignbyte(sdw(D, i + 1, a), lo, (uint32_t)a.qb);
}

// Header facts of the packet whose chunk run starts with v[0..5]; `act`
// marks the lanes whose result is used (wave-uniform paths consult only them).
// The header zone spans chunks 0..5; with NV = 4 loaded chunks, chunks 4..5
// are fetched (from c0, nch) only when some active packet has ip_hl != 5 —
// ip_hl 5 with both fields stays within bytes [q, q + 40) <= chunk 3.
template <int NV, bool NT>
__device__ __forceinline__ Hdr header(const uint4 (&v)[NV], const uint4 *c0, int nch, int q, int len,
				      uint32_t flags, bool act)
{
	static_assert(NV >= 4, "ip_hl 5 needs chunks 0..3");
	uint32_t D[24];
#pragma unroll
	for (int i = 0; i < 6; ++i) {
		const uint4 c = i < NV ? v[i < NV ? i : 0] : make_uint4(0, 0, 0, 0);
		D[4 * i + 0] = c.x;
		D[4 * i + 1] = c.y;
		D[4 * i + 2] = c.z;
		D[4 * i + 3] = c.w;
	}
	Align a;
	const int qd = q >> 2;
	a.qb = q & 3;
	a.shifted = __any(act && qd != 0);
	a.unaligned = __any(act && a.qb != 0);
	a.m1 = opaque((qd & 1) ? ~0u : 0u);
	a.m2 = opaque((qd & 2) ? ~0u : 0u);

	Hdr h;
	const uint32_t R0 = rdw(D, 0, a), R1 = rdw(D, 1, a), R2 = rdw(D, 2, a);
	const uint32_t R3 = rdw(D, 3, a), R4 = rdw(D, 4, a);
	h.hd = R0 & 15;
	h.proto = (R2 >> 8) & 0xffu;
	h.fip = R2 >> 16;
	h.ps = hsum(R4, hsum(R3, 0));
	const bool all5 = !__any(act && h.hd != 5);
	uint32_t hor = 5;
	if (!all5 && NV < 6) {
#pragma unroll
		for (int i = NV; i < 6; ++i) {
			const uint4 c = act && i < nch ? ld<NT>(c0 + i) : make_uint4(0, 0, 0, 0);
			D[4 * i + 0] = c.x;
			D[4 * i + 1] = c.y;
			D[4 * i + 2] = c.z;
			D[4 * i + 3] = c.w;
		}
	}
	if (all5) {
		h.ip = hsum(R4, hsum(R3, hsum(R2, hsum(R1, hsum(R0, 0)))));
	} else {
		// wave-uniform bound on the header dwords any lane needs (OR >= max)
		hor = 0;
#pragma unroll
		for (int b = 0; b < 4; ++b)
			hor |= __any(act && ((h.hd >> b) & 1)) ? (1u << b) : 0u;
		h.ip = hsum(h.hd > 4 ? R4 : 0u,
			    hsum(h.hd > 3 ? R3 : 0u,
				 hsum(h.hd > 2 ? R2 : 0u, hsum(h.hd > 1 ? R1 : 0u, hsum(h.hd > 0 ? R0 : 0u, 0)))));
#pragma unroll
		for (int i = 5; i < 15; ++i)
			if (i < (int)hor)
				h.ip = hsum((uint32_t)i < h.hd ? rdw(D, i, a) : 0u, h.ip);
	}
	h.fo = -1;
	h.fl4 = 0;
	const bool need_f = (flags & (CGCK_VERIFY | CGCK_ZERO_FIELDS | CGCK_STORE)) && (flags & CGCK_L4);
	if (need_f) {
		const int hl = (int)h.hd * 4;
		if (len >= 20 && len >= hl) {
			const int f = l4_field(h.proto, flags);
			if (f >= 0 && hl + f + 2 <= len)
				h.fo = f;
		}
		const int fi = h.fo >= 0 ? (hl + h.fo) >> 2 : -1; // dword of the field
		uint32_t fw = 0;
		if (all5) {
			// ip_hl 5: ICMP +2 -> dword 5, UDP +6 -> dword 6, TCP +16 -> dword 9
			const uint32_t R5 = rdw(D, 5, a), R6 = rdw(D, 6, a), R9 = rdw(D, 9, a);
			fw = fi == 9 ? R9 : (fi == 6 ? R6 : R5);
		} else {
#pragma unroll
			for (int i = 0; i < 20; ++i)
				if (i < (int)hor + 5)
					fw = i == fi ? rdw(D, i, a) : fw;
		}
		h.fl4 = (h.fo & 2) ? (fw >> 16) : (fw & 0xffffu);
	}
	return h;
}

// Bytes [0, q) of a chunk (before the packet), dword fast path when every
// active lane is dword aligned.
__device__ __forceinline__ uint32_t lead_sum(const uint4 &c, int q, bool dw)
{
	if (dw) {
		const int qd = q >> 2;
		return hsum(qd > 2 ? c.z : 0u, hsum(qd > 1 ? c.y : 0u, hsum(qd > 0 ? c.x : 0u, 0)));
	}
	return msum(c, 0, 0, q, 0);
}

// Bytes [e, 16) of a chunk (after the packet).
__device__ __forceinline__ uint32_t trail_sum(const uint4 &c, int e, bool dw)
{
	if (dw) {
		const int ed = e >> 2;
		return hsum(ed < 1 ? c.x : 0u, hsum(ed < 2 ? c.y : 0u, hsum(ed < 3 ? c.z : 0u, hsum(ed < 4 ? c.w : 0u, 0))));
	}
	return msum(c, 0, e, 16, 0);
}

// chunk j (0..7) of w[], no dynamic register index
__device__ __forceinline__ uint4 pick8(const uint4 (&w)[8], int j)
{
	const uint32_t b0 = opaque((j & 1) ? ~0u : 0u), b1 = opaque((j & 2) ? ~0u : 0u),
		       b2 = opaque((j & 4) ? ~0u : 0u);
	uint4 r;
#define CGCK_PICK8(f)                                                                          \
	r.f = pick(b2, pick(b1, pick(b0, w[7].f, w[6].f), pick(b0, w[5].f, w[4].f)),            \
		   pick(b1, pick(b0, w[3].f, w[2].f), pick(b0, w[1].f, w[0].f)))
	CGCK_PICK8(x);
	CGCK_PICK8(y);
	CGCK_PICK8(z);
	CGCK_PICK8(w);
#undef CGCK_PICK8
	return r;
}

// Finish one packet: T = folded sum over [ip, ip+len) in the ABSOLUTE frame.
__device__ __forceinline__ void finish(const KParams &p, uint64_t k, uint64_t a0, int len, uint32_t T,
				       const Hdr &h)
{
	const uint32_t flags = p.flags;
	if (a0 & 1)
		T = bswap16(T); // packet-relative
	uint32_t lo = 0, hi = 0, verdict = 0;
	const int hl = (int)h.hd * 4;
	if (flags & CGCK_RAW) {
		lo = finish(T);
	} else if (len < 20 || len < hl) {
		verdict = CGCK_BAD_LEN;
	} else {
		uint32_t IPs = fold16(h.ip), PS = fold16(h.ps);
		if (flags & (CGCK_ZERO_FIELDS | CGCK_VERIFY)) {
			T = ocsub(T, h.fip);
			if (hl >= 12)
				IPs = ocsub(IPs, h.fip);
			if (h.fo >= 0) {
				const int o = hl + h.fo;
				if (o != 10)
					T = ocsub(T, h.fl4);
				if (o >= 12 && o < 20)
					PS = ocsub(PS, h.fl4);
			}
		}
		if (flags & CGCK_IP)
			lo = finish(IPs);
		if (flags & CGCK_L4) {
			uint32_t L = ocsub(T, IPs);
			if (!(flags & CGCK_L4_NOPSEUDO))
				L = fold16(L + PS + (h.proto << 8) + bswap16((uint32_t)(len - hl) & 0xffffu));
			hi = finish(L);
		}
		if (flags & CGCK_VERIFY) {
			uint32_t want = h.fip;
			if ((flags & CGCK_V_IP_ZERO_IS_FFFF) && want == 0)
				want = 0xffffu;
			if ((flags & CGCK_IP) && lo != want)
				verdict |= CGCK_BAD_IP;
			if ((flags & CGCK_L4) && h.fo >= 0 &&
			    !((flags & CGCK_V_UDP_ZERO_SKIP) && h.proto == 17 && h.fl4 == 0) && hi != h.fl4)
				verdict |= CGCK_BAD_L4;
		}
		if (flags & CGCK_STORE) {
			uint8_t *ipp = reinterpret_cast<uint8_t *>(a0);
			if (flags & CGCK_IP)
				store16(ipp + 10, lo);
			if ((flags & CGCK_L4) && h.fo >= 0)
				store16(ipp + hl + h.fo, hi);
		}
	}
	if (p.out)
		gbl(p.out)[k] = lo | (hi << 16);
	if (p.verdict)
		gbl(p.verdict)[k] = (uint8_t)verdict;
	if (p.bad) {
		if (verdict & CGCK_BAD_IP)
			atomicAdd(p.bad + 0, 1u);
		if (verdict & CGCK_BAD_L4)
			atomicAdd(p.bad + 1, 1u);
	}
}

__device__ __forceinline__ int nchunks(uint64_t a0, uint32_t len)
{
	return len ? (int)(((a0 + len + 15) >> 4) - (a0 >> 4)) : 0;
}

// --------------------------------------------------------------------------
// Lane per packet
// --------------------------------------------------------------------------

template <bool DESC, bool NT, int S0, bool CLAMP>
__global__ __launch_bounds__(256) void lpp_kernel(KParams p)
{
	const bool raw = p.flags & CGCK_RAW;
	const Sched sc = sched((p.n + 255) / 256, p.contig);
	for (uint64_t it = sc.it; it < sc.end; it += sc.step) {
		const uint64_t k = it * 256 + threadIdx.x;
		const Pkt pk = get_pkt<DESC>(p, k);
		const uint64_t a0 = pk.a0;
		const int len = (int)pk.len, q = (int)(a0 & 15), nch = nchunks(a0, pk.len);
		const uint4 *c0 = reinterpret_cast<const uint4 *>(a0 & ~(uint64_t)15);
		// first S0 chunks: clamped and branch-free (precise vmcnt) or
		// predicated per lane (no duplicate loads)
		uint4 v[S0];
#pragma unroll
		for (int i = 0; i < S0; ++i)
			v[i] = CLAMP ? ldc<NT>(c0, i, nch, p.zero) : (i < nch ? ld<NT>(c0 + i) : make_uint4(0, 0, 0, 0));
		const bool more = __any(nch > S0);
		uint4 last = make_uint4(0, 0, 0, 0);
		if (CLAMP) {
			if (more)
				last = ldc<NT>(c0, nch - 1, nch, p.zero);
		} else {
			last = nch > S0 ? ld<NT>(c0 + nch - 1) : make_uint4(0, 0, 0, 0);
		}

		uint32_t tot = 0;
#pragma unroll
		for (int i = 0; i < S0; ++i)
			tot = i < nch ? sum4(v[i], tot) : tot;
		Hdr h{};
		if (!raw)
			h = header<S0, NT>(v, c0, nch, q, len, p.flags, pk.ok);
		if (more) {
			// chunks S0 .. nch-2 (the last one is `last`), 8 per step
			for (int t = S0; __any(t < nch - 1); t += 8) {
				uint4 w[8];
#pragma unroll
				for (int i = 0; i < 8; ++i)
					w[i] = t + i < nch - 1 ? ld<NT>(c0 + t + i) : make_uint4(0, 0, 0, 0);
				uint32_t s = 0;
#pragma unroll
				for (int i = 0; i < 8; ++i)
					s = sum4(w[i], s);
				tot = fold16(tot) + fold16(s);
			}
		}
		const bool dw = !__any(((q | len) & 3) != 0);
		if (__any(q != 0))
			tot = fold16(tot) + (0xffffu - fold16(lead_sum(v[0], q, dw)));
		const int e = q + len - 16 * (nch - 1); // bytes of the last chunk inside
		if (more)
			tot = fold16(tot) + fold16(nch > S0 ? sum4(last, 0) - trail_sum(last, e, dw) : 0u);
		if (__any(nch > 0 && nch <= S0 && e != 16)) {
			uint4 lc = make_uint4(0, 0, 0, 0);
#pragma unroll
			for (int i = 0; i < S0; ++i)
				if (i == nch - 1)
					lc = v[i];
			tot = fold16(tot) + (0xffffu - fold16(nch > 0 && nch <= S0 ? trail_sum(lc, e, dw) : 0u));
		}
		if (pk.ok)
			finish(p, k, a0, len, fold16(tot), h);
	}
}

// Software-pipelined lane-per-packet: while iteration i is computed, the
// chunks of iteration i+1 are already in flight (and, for descriptor
// batches, the descriptors of iteration i+2), so a wave never waits for
// memory between iterations.  Small packets only (nch <= S0 + the last
// chunk; longer packets take the same streaming loop as lpp_kernel).
template <bool DESC, bool NT>
__global__ __launch_bounds__(256) void lppp_kernel(KParams p)
{
	constexpr int S0 = 6;
	const bool raw = p.flags & CGCK_RAW;
	const Sched sc = sched((p.n + 255) / 256, p.contig);
	uint64_t it = sc.it;
	if (it >= sc.end)
		return;
	// prologue: descriptors of it and it+step, chunks of it
	Pkt pk = get_pkt<DESC>(p, it * 256 + threadIdx.x);
	Pkt pk2 = get_pkt<DESC>(p, (it + sc.step) * 256 + threadIdx.x);
	uint4 v[S0], last;
	{
		const int nch = nchunks(pk.a0, pk.len);
		const uint4 *c0 = reinterpret_cast<const uint4 *>(pk.a0 & ~(uint64_t)15);
#pragma unroll
		for (int i = 0; i < S0; ++i)
			v[i] = ldc<NT>(c0, i, nch, p.zero);
		last = ldc<NT>(c0, nch - 1, nch, p.zero);
	}
	for (; it < sc.end; it += sc.step) {
		const uint64_t k = it * 256 + threadIdx.x;
		// issue the next iteration's chunks (its descriptor is pk2)
		const Pkt pkn = pk2;
		uint4 vn[S0], lastn;
		{
			const int nch = nchunks(pkn.a0, pkn.len);
			const uint4 *c0 = reinterpret_cast<const uint4 *>(pkn.a0 & ~(uint64_t)15);
#pragma unroll
			for (int i = 0; i < S0; ++i)
				vn[i] = ldc<NT>(c0, i, nch, p.zero);
			lastn = ldc<NT>(c0, nch - 1, nch, p.zero);
		}
		pk2 = get_pkt<DESC>(p, (it + 2 * sc.step) * 256 + threadIdx.x);

		const uint64_t a0 = pk.a0;
		const int len = (int)pk.len, q = (int)(a0 & 15), nch = nchunks(a0, pk.len);
		const uint4 *c0 = reinterpret_cast<const uint4 *>(a0 & ~(uint64_t)15);
		uint32_t tot = 0;
#pragma unroll
		for (int i = 0; i < S0; ++i)
			tot = i < nch ? sum4(v[i], tot) : tot;
		Hdr h{};
		if (!raw)
			h = header<S0, NT>(v, c0, nch, q, len, p.flags, pk.ok);
		for (int t = S0; __any(t < nch - 1); t += 8) {
			uint4 w[8];
#pragma unroll
			for (int i = 0; i < 8; ++i)
				w[i] = t + i < nch - 1 ? ld<NT>(c0 + t + i) : make_uint4(0, 0, 0, 0);
			uint32_t s = 0;
#pragma unroll
			for (int i = 0; i < 8; ++i)
				s = sum4(w[i], s);
			tot = fold16(tot) + fold16(s);
		}
		const bool dw = !__any(((q | len) & 3) != 0);
		if (__any(q != 0))
			tot = fold16(tot) + (0xffffu - fold16(lead_sum(v[0], q, dw)));
		const int e = q + len - 16 * (nch - 1);
		if (__any(nch > S0))
			tot = fold16(tot) + fold16(nch > S0 ? sum4(last, 0) - trail_sum(last, e, dw) : 0u);
		if (__any(nch > 0 && nch <= S0 && e != 16)) {
			uint4 lc = make_uint4(0, 0, 0, 0);
#pragma unroll
			for (int i = 0; i < S0; ++i)
				if (i == nch - 1)
					lc = v[i];
			tot = fold16(tot) + (0xffffu - fold16(nch > 0 && nch <= S0 ? trail_sum(lc, e, dw) : 0u));
		}
		if (pk.ok)
			finish(p, k, a0, len, fold16(tot), h);
		pk = pkn;
#pragma unroll
		for (int i = 0; i < S0; ++i)
			v[i] = vn[i];
		last = lastn;
	}
}

// --------------------------------------------------------------------------
// Lane per 128-byte slot
// --------------------------------------------------------------------------

// inclusive prefix sum over the wave (values small enough for u32)
__device__ __forceinline__ uint32_t wave_scan(uint32_t x)
{
	const int l = threadIdx.x & 63;
#pragma unroll
	for (int d = 1; d < 64; d <<= 1) {
		const uint32_t y = __shfl_up(x, d, 64);
		if (l >= d)
			x += y;
	}
	return x;
}

__device__ __forceinline__ uint64_t shfl64(uint64_t x, int src)
{
	const uint32_t lo = __shfl((uint32_t)x, src, 64), hi = __shfl((uint32_t)(x >> 32), src, 64);
	return ((uint64_t)hi << 32) | lo;
}

// One window of up to 64 slots of ONE packet (jumbo packets, > 64 slots):
// returns the window's contribution (folded) on every lane.
template <bool NT>
__device__ __forceinline__ uint32_t jumbo_window(const uint4 *c0, int nch, int s, uint4 (&w)[8])
{
#pragma unroll
	for (int i = 0; i < 8; ++i)
		w[i] = 8 * s + i < nch ? ld<NT>(c0 + 8 * s + i) : make_uint4(0, 0, 0, 0);
	uint32_t r = 0;
#pragma unroll
	for (int i = 0; i < 8; ++i)
		r = sum4(w[i], r);
	return r;
}

template <bool DESC, bool NT>
__global__ __launch_bounds__(256) void slot_kernel(KParams p)
{
	__shared__ uint32_t mark[4][64];
	const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
	const bool raw = p.flags & CGCK_RAW;
	const uint64_t nwaves = (uint64_t)gridDim.x * 4;
	const uint64_t wid = (uint64_t)blockIdx.x * 4 + wv;
	const uint64_t per = (p.n + nwaves - 1) / nwaves;
	const uint64_t r0 = wid * per;
	const uint64_t r1 = r0 + per < p.n ? r0 + per : p.n;

	for (uint64_t cur = r0; cur < r1;) {
		// -- this iteration's packets and their slots --
		const uint64_t kk = cur + l;
		const Pkt pk = get_pkt<DESC>(p, kk < r1 ? kk : p.n); // past the range: !ok
		const int nch_l = nchunks(pk.a0, pk.len);
		const uint32_t ns = pk.ok ? (uint32_t)max(1, (nch_l + 7) >> 3) : 0u;
		const uint32_t P = wave_scan(ns);
		const uint64_t fit = __ballot(pk.ok && P <= 64);
		const int m = __popcll(fit);

		if (m == 0) {
			// Jumbo packet (> 64 slots): windows of 64 slots, whole-wave sums.
			const uint64_t a0 = shfl64(pk.a0, 0);
			const int len = __shfl((int)pk.len, 0, 64), nch = __shfl(nch_l, 0, 64);
			const int q = (int)(a0 & 15);
			const uint4 *c0 = reinterpret_cast<const uint4 *>(a0 & ~(uint64_t)15);
			const int nsj = (nch + 7) >> 3;
			uint32_t acc = 0;
			Hdr h{};
			for (int wbase = 0; wbase < nsj; wbase += 64) {
				const int s = wbase + l;
				uint4 w[8];
				uint32_t r = jumbo_window<NT>(c0, nch, s, w);
				if (wbase == 0 && !raw)
					h = header<8, NT>(w, c0, nch, q, len, p.flags, l == 0);
				const int j = (nch - 1) - 8 * s; // last chunk's position in this slot
				const int e = q + len - 16 * (nch - 1);
				uint32_t corr = 0;
				if (s == 0 && q != 0)
					corr += lead_sum(w[0], q, false);
				if (j >= 0 && j < 8 && e != 16)
					corr += trail_sum(pick8(w, j), e, false);
				r = fold16(r) + (0xffffu - fold16(corr));
				acc = fold16(acc) + fold16(gsum<64>(r));
			}
			if (l == 0)
				finish(p, cur, a0, len, fold16(acc), h);
			cur += 1;
			continue;
		}

		// -- lane -> (owner packet, slot) through per-wave head markers --
		const int T = __shfl((int)P, m - 1, 64); // slots in use
		const int st = (int)(P - ns);            // first slot of lane l's packet
		mark[wv][l] = 0;
		__builtin_amdgcn_wave_barrier();
		asm volatile("" ::: "memory");
		if (l < m)
			mark[wv][st] = 1;
		__builtin_amdgcn_wave_barrier();
		asm volatile("" ::: "memory");
		const uint32_t hf = mark[wv][l];
		const uint64_t heads = __ballot(hf != 0 && l < T);
		const uint64_t le = l == 63 ? ~0ull : ((2ull << l) - 1);
		const int owner = max(0, __popcll(heads & le) - 1);
		const bool act = l < T;

		const uint64_t a0 = shfl64(pk.a0, owner);
		const int len = __shfl((int)pk.len, owner, 64);
		const int nch = __shfl(nch_l, owner, 64);
		const int st_o = __shfl(st, owner, 64);
		const int ns_o = __shfl((int)ns, owner, 64);
		const int s = l - st_o; // slot index inside the packet
		const int q = (int)(a0 & 15);
		const uint4 *c0 = reinterpret_cast<const uint4 *>(a0 & ~(uint64_t)15);

		// clamped, branch-free: slot tails and idle lanes re-read the
		// packet's last chunk (or the zero chunk) and are dropped below
		uint4 w[8];
#pragma unroll
		for (int i = 0; i < 8; ++i)
			w[i] = ldc<NT>(c0, 8 * s + i, act ? nch : 0, p.zero);
		uint32_t r = 0;
#pragma unroll
		for (int i = 0; i < 8; ++i)
			r = act && 8 * s + i < nch ? sum4(w[i], r) : r;

		const bool head = act && s == 0;
		Hdr h{};
		if (!raw)
			h = header<8, NT>(w, c0, nch, q, len, p.flags, head);

		// edges: lead on the head lane, trail on the lane holding chunk nch-1
		const bool dw = !__any(act && ((q | len) & 3) != 0);
		uint32_t corr = 0;
		if (__any(head && q != 0))
			corr = head && q != 0 ? lead_sum(w[0], q, dw) : 0u;
		const int j = (nch - 1) - 8 * s;
		const int e = q + len - 16 * (nch - 1);
		const bool tail = act && nch > 0 && j >= 0 && j < 8 && e != 16;
		if (__any(tail))
			corr += tail ? trail_sum(pick8(w, j), e, dw) : 0u;
		r = fold16(r) + (0xffffu - fold16(corr));

		// segmented suffix sum towards the head lane
		uint32_t nso = 0; // wave-uniform bound on segment length (OR >= max)
#pragma unroll
		for (int b = 0; b < 7; ++b)
			nso |= __any(act && ((ns_o >> b) & 1)) ? (1u << b) : 0u;
		const int send = st_o + ns_o;
#pragma unroll
		for (int d = 1; d < 64; d <<= 1) {
			if ((uint32_t)d >= nso)
				break;
			const uint32_t y = __shfl_down(r, d, 64);
			if (l + d < send)
				r += y;
		}
		if (head)
			finish(p, cur + owner, a0, len, fold16(r), h);
		cur += m;
	}
}

// --------------------------------------------------------------------------
// Launchers
// --------------------------------------------------------------------------

template <bool DESC, int S0, bool CLAMP>
static hipError_t launch_lpp_t(const KParams &p, int max_blocks, bool nt, hipStream_t st)
{
	uint64_t want = (p.n + 255) / 256;
	int blocks = (int)(want < (uint64_t)max_blocks ? want : (uint64_t)max_blocks);
	if (blocks < 1)
		blocks = 1;
	if (nt)
		hipLaunchKernelGGL((lpp_kernel<DESC, true, S0, CLAMP>), dim3(blocks), dim3(256), 0, st, p);
	else
		hipLaunchKernelGGL((lpp_kernel<DESC, false, S0, CLAMP>), dim3(blocks), dim3(256), 0, st, p);
	return hipGetLastError();
}

template <bool DESC>
static hipError_t launch_slot_t(const KParams &p, int max_blocks, bool nt, hipStream_t st)
{
	// each wave owns a contiguous packet range of >= ~64 packets
	uint64_t want = (p.n + 4 * 64 - 1) / (4 * 64);
	int blocks = (int)(want < (uint64_t)max_blocks ? want : (uint64_t)max_blocks);
	if (blocks < 1)
		blocks = 1;
	if (nt)
		hipLaunchKernelGGL((slot_kernel<DESC, true>), dim3(blocks), dim3(256), 0, st, p);
	else
		hipLaunchKernelGGL((slot_kernel<DESC, false>), dim3(blocks), dim3(256), 0, st, p);
	return hipGetLastError();
}

template <bool DESC>
static hipError_t launch_lppp_t(const KParams &p, int max_blocks, bool nt, hipStream_t st)
{
	uint64_t want = (p.n + 255) / 256;
	int blocks = (int)(want < (uint64_t)max_blocks ? want : (uint64_t)max_blocks);
	if (blocks < 1)
		blocks = 1;
	if (nt)
		hipLaunchKernelGGL((lppp_kernel<DESC, true>), dim3(blocks), dim3(256), 0, st, p);
	else
		hipLaunchKernelGGL((lppp_kernel<DESC, false>), dim3(blocks), dim3(256), 0, st, p);
	return hipGetLastError();
}

hipError_t launch_lppp(const KParams &p, int num_cus, bool nt, hipStream_t st)
{
	return p.desc ? launch_lppp_t<true>(p, num_cus * 8, nt, st) : launch_lppp_t<false>(p, num_cus * 8, nt, st);
}

// shape: 0 = 4 chunks up front, clamped; 1 = 6 clamped; 2 = 6 predicated;
// 3 = 4 predicated
hipError_t launch_lpp(const KParams &p, int num_cus, bool nt, int shape, hipStream_t st)
{
	const int mb = num_cus * 8;
	const bool d = p.desc != nullptr;
	switch (shape) {
	case 1:
		return d ? launch_lpp_t<true, 6, true>(p, mb, nt, st) : launch_lpp_t<false, 6, true>(p, mb, nt, st);
	case 2:
		return d ? launch_lpp_t<true, 6, false>(p, mb, nt, st) : launch_lpp_t<false, 6, false>(p, mb, nt, st);
	case 3:
		return d ? launch_lpp_t<true, 4, false>(p, mb, nt, st) : launch_lpp_t<false, 4, false>(p, mb, nt, st);
	default:
		return d ? launch_lpp_t<true, 4, true>(p, mb, nt, st) : launch_lpp_t<false, 4, true>(p, mb, nt, st);
	}
}

hipError_t launch_slot(const KParams &p, int num_cus, bool nt, hipStream_t st)
{
	return p.desc ? launch_slot_t<true>(p, num_cus * 8, nt, st) : launch_slot_t<false>(p, num_cus * 8, nt, st);
}

} // namespace cgck
