// cgck_lane.h — per-packet device helpers shared by the lane kernels
// (cgck_lane.hip) and the packed-span kernel (cgck_span.hip): header facts
// from a packet's first chunks, edge corrections, the result() finish
// (zero-field semantics, pseudo-header, reduce() of subr.c:137-156, verdicts,
// stores), output staging, descriptor decoding and wave scans.
#pragma once
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

// One packet's outputs: the u32 (ip | l4 << 16) and the verdict byte.
struct Res {
	uint32_t out, verdict;
};

// Finish one packet: T = folded sum over [ip, ip+len) in the ABSOLUTE frame.
// In-place field stores (CGCK_STORE) and the bad counters happen here; the
// per-packet outputs are returned for the caller to emit (or stage).
__device__ __forceinline__ Res result(const KParams &p, uint64_t a0, int len, uint32_t T, const Hdr &h)
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
	if (p.bad) {
		if (verdict & CGCK_BAD_IP)
			atomicAdd(p.bad + 0, 1u);
		if (verdict & CGCK_BAD_L4)
			atomicAdd(p.bad + 1, 1u);
	}
	return Res{lo | (hi << 16), verdict};
}

__device__ __forceinline__ void emit(const KParams &p, uint64_t k, const Res &r)
{
	if (p.out)
		gbl(p.out)[k] = r.out;
	if (p.verdict)
		gbl(p.verdict)[k] = (uint8_t)r.verdict;
}

__device__ __forceinline__ void finish(const KParams &p, uint64_t k, uint64_t a0, int len, uint32_t T,
				       const Hdr &h)
{
	emit(p, k, result(p, a0, len, T, h));
}

// --------------------------------------------------------------------------
// Output staging
// --------------------------------------------------------------------------
//
// On gfx9 vmcnt counts stores as well as loads and retires in order, so a
// per-iteration output store makes the NEXT iteration's wait for its loads
// also wait for that store's write acknowledgement — measured at -20% of
// the stream rate on 64 B packets and IMIX for ~1% of the bytes.  Outputs
// of the slot kernels (scattered head-lane stores, ~20 per iteration) are
// therefore staged in LDS and written in coalesced bursts: one exposed store
// latency per window instead of per iteration.  (For grid-stride lane per
// packet, whose stores are already coalesced, a burst of 8 measured worse
// than one store per iteration: 58.5% vs 65.5% of HBM peak on 64 B.)

// Lane per slot: a window of kWaveStage consecutive packets of the wave's
// range [sb, sb + kWaveStage), written by head lanes, flushed by all lanes
// with nontemporal stores.  2048-packet windows (40 KiB of LDS per block, 4
// blocks per CU) against 256: +9.8 % on IMIX in the same process, 1024 with
// nt +4-5 %, nt alone at 256 nothing (tools/ab_inproc.py,
// profiles/r01/ab_slot_window.log): each flush's stores stall the next loads
// once (in-order vmcnt), so fewer, longer flushes.
constexpr int kWaveStage = 2048;

struct WaveStage {
	uint32_t *so;
	uint8_t *sv;
	uint64_t sb;
};

__device__ __forceinline__ void wave_stage_flush(const KParams &p, WaveStage &s, uint64_t e)
{
	const int l = threadIdx.x & 63;
	__builtin_amdgcn_wave_barrier();
	asm volatile("" ::: "memory");
	const int c = (int)(e - s.sb);
	if (p.out)
		flush_u32(s.so, p.out + s.sb, c, l, 64);
	if (p.verdict)
		for (int i = l; i < c; i += 64)
			gbl(p.verdict)[s.sb + i] = s.sv[i];
	__builtin_amdgcn_wave_barrier();
	asm volatile("" ::: "memory");
	s.sb = e;
}

// make room for packets [cur, cur + m)
__device__ __forceinline__ void wave_stage_reserve(const KParams &p, WaveStage &s, uint64_t cur, int m)
{
	if (cur + m > s.sb + kWaveStage)
		wave_stage_flush(p, s, cur);
}

__device__ __forceinline__ void wave_stage_put(WaveStage &s, uint64_t k, const Res &r)
{
	s.so[k - s.sb] = r.out;
	s.sv[k - s.sb] = (uint8_t)r.verdict;
}

__device__ __forceinline__ int nchunks(uint64_t a0, uint32_t len)
{
	return len ? (int)(((a0 + len + 15) >> 4) - (a0 >> 4)) : 0;
}

__device__ __forceinline__ uint64_t shfl64(uint64_t x, int src)
{
	const uint32_t lo = __shfl((uint32_t)x, src, 64), hi = __shfl((uint32_t)(x >> 32), src, 64);
	return ((uint64_t)hi << 32) | lo;
}

// x of lane `src` (wave-uniform), in SGPRs: readlane instead of a shuffle,
// so values derived from it stay scalar (uniform loop bounds, branches)
__device__ __forceinline__ uint64_t readlane64(uint64_t x, int src)
{
	const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, src);
	const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), src);
	return ((uint64_t)hi << 32) | lo;
}

struct DescW {
	uint32_t lo, hi, w2;
};

// descriptor words of packet k (k past the wave's range reads packet 0)
template <bool DESC>
__device__ __forceinline__ DescW load_desc(const KParams &p, uint64_t k, uint64_t r1)
{
	DescW d{0, 0, 0};
	if (DESC) {
		const CGCK_GLOBAL uint32_t *q = (const CGCK_GLOBAL uint32_t *)p.desc + 3 * (k < r1 ? k : 0);
		d.lo = q[0];
		d.hi = q[1];
		d.w2 = q[2];
	}
	return d;
}

template <bool DESC>
__device__ __forceinline__ Pkt decode(const KParams &p, uint64_t k, uint64_t r1, const DescW &d)
{
	Pkt r;
	r.ok = k < r1;
	if (DESC) {
		r.a0 = reinterpret_cast<uint64_t>(p.base) + (((uint64_t)d.hi << 32) | d.lo) + (d.w2 & 0xffffu);
		r.len = d.w2 >> 16;
	} else {
		r.a0 = reinterpret_cast<uint64_t>(p.base) + (r.ok ? k : 0) * p.stride + p.l3_off;
		r.len = p.ip_len;
	}
	if (!r.ok)
		r.len = 0;
	return r;
}

// inclusive prefix sum over the wave in DPP (row shifts, then the row
// broadcasts of lanes 15 and 31); no LDS round trips
__device__ __forceinline__ uint32_t wave_scan_dpp(uint32_t x)
{
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false); // row_shr:1
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false); // row_shr:2
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false); // row_shr:4
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false); // row_shr:8
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false); // row_bcast:15
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false); // row_bcast:31
	return x;
}

// inclusive max-scan over the wave in DPP (same pattern as wave_scan_dpp;
// lanes whose DPP source is out of range read 0, which max leaves alone)
__device__ __forceinline__ uint32_t wave_max_scan_dpp(uint32_t x)
{
#define CGCK_MAXDPP(ctrl, rmask)                                                                         \
	{                                                                                                \
		const uint32_t y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, ctrl, rmask, 0xf, false); \
		x = y > x ? y : x;                                                                       \
	}
	CGCK_MAXDPP(0x111, 0xf) // row_shr:1
	CGCK_MAXDPP(0x112, 0xf) // row_shr:2
	CGCK_MAXDPP(0x114, 0xf) // row_shr:4
	CGCK_MAXDPP(0x118, 0xf) // row_shr:8
	CGCK_MAXDPP(0x142, 0xa) // row_bcast:15
	CGCK_MAXDPP(0x143, 0xc) // row_bcast:31
#undef CGCK_MAXDPP
	return x;
}

} // namespace cgck
