// cgck_group.hip — the lane-group kernel: G lanes own one packet and walk
// its 16-byte chunks with coalesced uint4 loads, S steps unrolled; group
// partials are reduced with DPP.  Used for large packets (>= 1 KiB, the
// 1500 B MTU configuration) and for the single-region drop-in calls.
//
// Per packet three masked sums are formed from one HBM stream:
//   tot = sum over [ip, ip+ip_len)           (all lanes)
//   ip  = sum over [ip, ip+ip_hl*4)          (header-zone lanes only)
//   ps  = sum over [ip+12, ip+20)            (src/dst of the pseudo-header)
// and the L4 sum is tot - ip (one's complement), plus ps, ip_p<<8 and
// htons(l4len) read as a little-endian word (struct pseudo, subr.c:119-125).
#include "cgck_device.h"

#include <stdlib.h>

namespace cgck {

// Part and eat(): cgck_device.h (shared with the LDS-DMA stream kernel).

// Per-packet outputs of a block with a contiguous range are staged in LDS
// and leave in windows of kGrpStage packets by nontemporal, fully coalesced
// stores: on gfx9 a store counts in vmcnt, which retires in order, so a
// store per iteration puts its write acknowledgement in front of the next
// iteration's loads (1500 B: 79.2 % of HBM peak with the per-packet store,
// 82.7 % with none).
constexpr int kGrpStage = 2048;

// LDSD: p.desc points at descriptors staged in LDS (the burst server's slices).
// SYS (U = 1, packets of at most S * G chunks): the packet bytes are host
// memory the burst server reads in place, with system-coherent loads
// (ld_sys16xN) instead of after a cache-invalidating acquire; the header
// bytes come from the chunks (lane shuffles) rather than byte loads.
// SYSST: every store is a system-coherent one (sc0 sc1, written through to
// host memory): the burst server's outputs and in-place fields, which it then
// publishes after the stores' own completion instead of an L2 write-back.
// LDSP: packet bytes in LDS (p.base and p.zero generic pointers into it).
// FL: the flags, known at compile time (0: p.flags, read at run time).
template <int G, int S, int U, bool DESC, bool NT, bool LDSD = false, bool SYS = false, bool SYSST = false,
	  bool LDSP = false, uint32_t FL = 0>
__device__ __forceinline__ void cksum_body(const KParams &p, uint32_t bid, uint32_t nb)
{
	__shared__ uint32_t so[kGrpStage];
	constexpr int GPB = 256 / G;        // groups per block
	constexpr int PPB = GPB * U;        // packets per block iteration
	const int lane = threadIdx.x;
	const int gib = lane / G;           // group in block
	const int gl = lane % G;            // lane in group
	const uint32_t flags = FL ? FL : p.flags;
	const bool raw = flags & CGCK_RAW;
	const bool need_hdr = !raw;
	const bool rx = flags & kFlagRx; // uniform

	const Sched sc = sched((p.n + PPB - 1) / PPB, p.contig, bid, nb);
	const bool stage = p.contig && p.out; // block-uniform
	uint64_t wb = sc.it * PPB;            // first packet of the open window
	auto flush = [&](uint64_t e) {        // block-uniform call
		__syncthreads();
		const uint64_t end = e < p.n ? e : p.n;
		if (end > wb)
			flush_u32(so, p.out + wb, (int)(end - wb), threadIdx.x, 256);
		__syncthreads();
		wb = e;
	};
	for (uint64_t blk = sc.it; blk < sc.end; blk += sc.step) {
		if (stage && (blk + 1) * PPB > wb + kGrpStage)
			flush(blk * PPB);
		Pkt pk[U];
		uint32_t b0[U], proto[U], tl[U]; // tl: ntohs(ip_len)'s bytes (kFlagRx)
		uint4 v[U][S];
		int nch[U];
#pragma unroll
		for (int u = 0; u < U; ++u) {
			if constexpr (LDSD)
				pk[u] = get_pkt_lds(p, blk * PPB + (uint64_t)u * GPB + gib);
			else
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
			tl[u] = 0;
			if (!SYS && need_hdr && pk[u].ok && span > 0) {
				b0[u] = ld8q<LDSP>(a0);
				if (span > 9)
					proto[u] = ld8q<LDSP>(a0 + 9);
				// kFlagRx: the frame's own length field, read with the
				// chunks (one round trip), so its coverage is decided after
				// the loads and the surplus chunks are masked by position
				if (rx && span >= 20)
					tl[u] = ld8q<LDSP>(a0 + 2) << 8 | ld8q<LDSP>(a0 + 3);
			}
			const uint4 *c0 = reinterpret_cast<const uint4 *>(a0 & ~(uint64_t)15);
			// clamped: chunks past the packet re-read its last chunk and
			// eat() masks them out by position (zero-chunk lanes read zeros)
			if constexpr (SYS) {
				static_assert(U == 1, "the system-coherent body runs one packet per group");
				const uint4 *a[S];
#pragma unroll
				for (int s = 0; s < S; ++s)
					a[s] = nch[u] > 0 ? c0 + min(s * G + gl, nch[u] - 1) : reinterpret_cast<const uint4 *>(p.zero);
				ld_sys16xN<S>(a, v[u]);
				// the header bytes at +0, +2, +3, +9 (aligned offsets q + k <
				// 32): chunk 0 or 1 of the packet, lane 0 or 1 of the group
				const int q = (int)(a0 & 15);
				const int base_lane = lane & 63 & ~(G - 1); // the group's first lane in the wave
				auto byte_at = [&](int k) {
					const int o = q + k;
					const uint4 w = v[u][0];
					const int di = (o & 15) >> 2;
					const uint32_t d = di == 0 ? w.x : di == 1 ? w.y : di == 2 ? w.z : w.w;
					return (uint32_t)__shfl((int)((d >> (8 * (o & 3))) & 0xffu), base_lane + (o >> 4), 64);
				};
				const uint32_t h0 = byte_at(0), h2 = byte_at(2), h3 = byte_at(3), h9 = byte_at(9);
				if (need_hdr && pk[u].ok && span > 0) {
					b0[u] = h0;
					if (span > 9)
						proto[u] = h9;
					if (rx && span >= 20)
						tl[u] = h2 << 8 | h3;
				}
			} else {
#pragma unroll
				for (int s = 0; s < S; ++s)
					v[u][s] = ldcq<NT, LDSP>(c0, s * G + gl, nch[u], p.zero);
			}
		}
#pragma unroll
		for (int u = 0; u < U; ++u) {
			const int q = (int)(pk[u].a0 & 15);
			uint32_t rxm = 0, cover = pk[u].len;
			if (rx)
				rxm = rx_meta(pk[u].len, b0[u], tl[u] >> 8, tl[u] & 0xffu, proto[u], &cover);
			const int len = (int)cover;
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
			// (Never with SYS: its caller keeps packets within S * G chunks.)
			const uint4 *c0 = reinterpret_cast<const uint4 *>(pk[u].a0 & ~(uint64_t)15);
			for (int s = S; __any(s * G < nch[u]); ++s) {
				const int k = s * G + gl;
				uint4 w = k < nch[u] ? ldq<NT, LDSP>(c0 + k) : make_uint4(0, 0, 0, 0);
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
					if (l4_nopseudo(proto[u], flags)) {
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
						store16p<SYSST>(ipp + 10, lo);
					if ((flags & CGCK_L4) && fo >= 0)
						store16p<SYSST>(ipp + hl + fo, hi);
				}
			}
			if (stage)
				so[k - wb] = lo | (hi << 16);
			else if (p.out)
				st32p<SYSST>(gbl(p.out) + k, lo | (hi << 16));
			if (p.verdict)
				st8p<SYSST>(gbl(p.verdict) + k, (uint8_t)verdict);
			if (rx && p.meta)
				st32p<SYSST>(gbl(p.meta) + k, rxm);
			if (p.bad) {
				if (verdict & CGCK_BAD_IP)
					atomicAdd(p.bad + 0, 1u);
				if (verdict & CGCK_BAD_L4)
					atomicAdd(p.bad + 1, 1u);
			}
		}
	}
	if (stage && sc.it < sc.end)
		flush(sc.end * PPB);
}

template <int G, int S, int U, bool DESC, bool NT>
__global__ __launch_bounds__(256) void cksum_kernel(KParams p)
{
	cksum_body<G, S, U, DESC, NT>(p, blockIdx.x, gridDim.x);
}

// --------------------------------------------------------------------------
// Burst server: K resident workgroups that serve small and mid-size
// host-resident batches (RX bursts, drop-in calls) without a launch or a
// stream synchronisation per batch.  The host writes a request block
// (BurstReq, descriptors, packet bytes) into host-coherent staging and stores
// req = seq | n << 32; thread 0 of workgroup 0 polls it with relaxed
// system-scope loads and relays it to the others.  W = burst_wgs(n, K)
// workgroups serve the request:
//  * W == 1 (up to kBurstOneWG packets: a drop-in call, a small burst):
//    workgroup 0 copies the block into device scratch with one wide read
//    (tools/pingpong: every dependent host round trip costs ~1.3 us, so the
//    block is fetched at once instead of header -> descriptor -> packet
//    bytes) and runs the group body over the copy, or over registered ring
//    memory in place;
//  * W > 1: workgroup j reads the header and its own slice of the
//    descriptors (d_off is fixed, so both in one round trip) into its LDS,
//    then the packet bytes where they lie (registered memory, or the block):
//    the burst's host reads spread over W CUs, as a launch's would.  No byte
//    of a slice passes through cached device memory.
// Before any packet load or store every serving workgroup checks the header
// and each of its descriptors: inside the block (staged bytes) or inside the
// request's `range` (registered memory read in place); a refused request
// counts in bad_req and its host call fails with -EIO.
// Each serving workgroup writes its outputs to host-coherent memory and
// publishes done[j] after a system-scope release.  Every poll loop is
// bounded: a workgroup exits on `stop`, or after idle_ticks of the 100 MHz
// real-time counter without a request (the host relaunches the server when
// it finds a workgroup gone), so no launch outlives its context.
//
// Ordering of the request block: the host's block stores precede its `req`
// store (x86 TSO, a release store); the block, the mailbox and the packet
// bytes are system memory, read with system-coherent loads (sc0 sc1:
// ld_sys16x2, sys_relaxed) or with plain loads after a system-scope acquire,
// so no line a cache holds from an earlier request is served.  A worker's block reads are issued after its relay load
// returned, the relay was stored after the leader's mailbox load returned the
// new seq, and that load was served after the host's block stores were
// visible: each read is causally after the block was written.  The
// whole-block path's device scratch copy is written and read by one
// workgroup: a workgroup-scope release / acquire around the barrier and an
// L1 invalidate, so no line of an earlier request's copy is served.
// --------------------------------------------------------------------------

__device__ __forceinline__ uint32_t sys_load(const uint32_t *p)
{
	return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint32_t sys_relaxed(const uint32_t *p)
{
	return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint64_t sys_relaxed64(const uint64_t *p)
{
	return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The group body over a request's packets [lo, hi) (block 0 of 1); desc is
// packet lo's descriptor (in LDS when LDSD); LDSP: the packet bytes too.
template <bool LDSD, bool SYS = false, bool LDSP = false, bool WT = true, uint32_t FL = 0>
__device__ __forceinline__ void burst_part(const BurstReq &h, uint32_t flags, const uint32_t *desc, uint32_t lo,
					   uint32_t hi, uint32_t *out, uint32_t *meta, uint8_t *verdict,
					   const void *zero, const uint8_t *base)
{
	KParams p = {base, reinterpret_cast<const cgck_desc_t *>(desc), hi - lo, 0, 0, 0, flags,
		     out ? out + lo : nullptr, verdict ? verdict + lo : nullptr, nullptr, 0, zero, meta + lo};
	// WT: the body's stores to host memory are system-coherent (SYSST),
	// published after their own completion (a one-workgroup request); a
	// wide request's slices store plainly and publish after an L2 write-back
	// (thousands of written-through 4-byte stores leave as as many fabric
	// writes: 2048 x 1500 B in place 79 -> 86 us, tools/e2e.py)
	if constexpr (SYS) { // burst_sys_ok: one packet per group covers the part
		if (h.max_len <= 80)
			cksum_body<4, 2, 1, true, false, LDSD, true, true, false, FL>(p, 0, 1);
		else
			cksum_body<16, 6, 1, true, false, LDSD, true, true, false, FL>(p, 0, 1);
		return;
	}
	if constexpr (LDSP) { // a block of <= 8 KiB: at most ~64 small packets
		if (h.max_len <= 80)
			cksum_body<4, 2, 1, true, false, LDSD, false, true, true, FL>(p, 0, 1);
		else
			cksum_body<16, 6, 1, true, false, LDSD, false, true, true, FL>(p, 0, 1);
		return;
	}
	// A part the block covers in one pass with one packet per group runs
	// unrolled once (U = 1): a small request's time is the body's dependent
	// VALU chain, which four unrolled packets per group quadruple.
	if (h.max_len <= 80) {
		if (hi - lo <= 64)
			cksum_body<4, 2, 1, true, false, LDSD, false, WT, false, FL>(p, 0, 1);
		else
			cksum_body<4, 2, 4, true, false, LDSD, false, WT, false, FL>(p, 0, 1);
	} else {
		if (hi - lo <= 16)
			cksum_body<16, 6, 1, true, false, LDSD, false, WT, false, FL>(p, 0, 1);
		else
			cksum_body<16, 6, 4, true, false, LDSD, false, WT, false, FL>(p, 0, 1);
	}
}

// A request may carry two parts (a receive burst's frames, then a TX fill's
// packets: BurstReq.n1): packets [lo, hi) on either side of n1 run with that
// part's flags.
template <bool LDSD, bool SYS = false, bool LDSP = false, bool WT = true, uint32_t FL = 0>
__device__ __forceinline__ void burst_body(const BurstReq &h, const uint32_t *desc, uint32_t lo, uint32_t hi,
					   uint32_t *out, uint32_t *meta, uint8_t *verdict, const void *zero,
					   const uint8_t *base)
{
	const uint32_t n1 = h.n1 < h.n ? h.n1 : 0;
	if (n1 > lo && n1 < hi) {
		burst_part<LDSD, SYS, LDSP, WT>(h, h.flags, desc, lo, n1, out, meta, verdict, zero, base);
		__syncthreads(); // (the body's LDS staging is reused)
		burst_part<LDSD, SYS, LDSP, WT>(h, h.flags2, desc + 3 * (n1 - lo), n1, hi, out, meta, verdict, zero, base);
	} else {
		burst_part<LDSD, SYS, LDSP, WT, FL>(h, n1 && lo >= n1 ? h.flags2 : h.flags, desc, lo, hi, out, meta,
						verdict, zero, base);
	}
}

// Lab A/B build (-DCGCK_SERVER_SMALL_ONLY=1): a server kernel with only the
// staged one-workgroup path (every other request refused) — how much of the
// small path's cost is the size of the function around it.
#if !CGCK_LAB || !defined(CGCK_SERVER_SMALL_ONLY)
#undef CGCK_SERVER_SMALL_ONLY
#define CGCK_SERVER_SMALL_ONLY 0
#endif

// burst_body for a one-workgroup request, compiled for the flag sets the
// library posts (FL: every flag test folds, 0.9-1.1 k of a small request's
// 2.2-4.3 k body cycles, tools/bodylat): the drop-in in_cksum / udp_cksum
// calls, the RX and TX windows' requests, cgck_desc_host's BSD verify and
// in-place fill; any other set, and a two-part request, take the run-time
// flags.
// (Lab opts bit 8192: the run-time flags for every request, the A/B.)
template <bool LDSD, bool SYS = false, bool LDSP = false>
__device__ __forceinline__ void burst_body_spec(const BurstReq &h, const uint32_t *desc, uint32_t n, uint32_t *out,
						uint32_t *meta, uint8_t *verdict, const void *zero, const uint8_t *base,
						uint32_t opts)
{
#if !CGCK_LAB
	(void)opts;
#else
	if (!(opts & 8192))
#endif
	if (!(h.n1 && h.n1 < h.n)) {
		switch (h.flags) {
		case kRxFlags:
			return burst_body<LDSD, SYS, LDSP, true, kRxFlags>(h, desc, 0, n, out, meta, verdict, zero, base);
		case kTxFlags:
			return burst_body<LDSD, SYS, LDSP, true, kTxFlags>(h, desc, 0, n, out, meta, verdict, zero, base);
		case kTxFlags | kFlagL4Auto:
			return burst_body<LDSD, SYS, LDSP, true, kTxFlags | kFlagL4Auto>(h, desc, 0, n, out, meta, verdict,
											  zero, base);
		case CGCK_VERIFY_BSD:
			return burst_body<LDSD, SYS, LDSP, true, CGCK_VERIFY_BSD>(h, desc, 0, n, out, meta, verdict, zero,
										  base);
		case CGCK_FILL_BOTH:
			return burst_body<LDSD, SYS, LDSP, true, CGCK_FILL_BOTH>(h, desc, 0, n, out, meta, verdict, zero,
										 base);
		}
		if constexpr (LDSP) { // the drop-in symbols' one region, staged
			if (h.flags == CGCK_RAW)
				return burst_body<LDSD, SYS, LDSP, true, CGCK_RAW>(h, desc, 0, n, out, meta, verdict, zero, base);
			if (h.flags == (CGCK_L4 | kFlagNoLenCheck))
				return burst_body<LDSD, SYS, LDSP, true, CGCK_L4 | kFlagNoLenCheck>(h, desc, 0, n, out, meta,
												     verdict, zero, base);
		}
	}
	burst_body<LDSD, SYS, LDSP>(h, desc, 0, n, out, meta, verdict, zero, base);
}

// Can a one-workgroup request of n packets read its packet bytes in place
// with the system-coherent body?  One packet per lane group must cover each
// part in one pass (64 groups of 4 lanes up to 80 bytes, 16 of 16 lanes
// above), with every packet within the body's S * G chunks (1536 bytes).
__device__ __forceinline__ bool burst_sys_ok(const BurstReq &h, uint32_t n)
{
	return h.max_len <= 80 ? n <= 64 : (n <= 16 && h.max_len <= 1520);
}

// A request header the server can serve: the count it was told, inside the
// context's capacity and block, descriptors where the host puts them, staged
// bytes inside the block.
__device__ __forceinline__ bool burst_hdr_ok(const BurstReq &h, uint32_t n, uint32_t max_pkts, uint32_t cap)
{
	return h.n == n && h.n <= max_pkts && h.bytes <= cap && h.d_off == sizeof(BurstReq) &&
	       (uint64_t)h.d_off + 12ull * h.n <= h.bytes && (h.base ? h.range != 0 : h.p_off <= h.bytes);
}

// Bytes a descriptor may reach from the packet base: the request's range in
// place, the staged bytes of the block otherwise (burst_hdr_ok held).
__device__ __forceinline__ uint64_t burst_limit(const BurstReq &h)
{
	return h.base ? h.range : (uint64_t)(h.bytes - h.p_off);
}

// Descriptors of one slice pass staged in LDS (12 KiB): a slice of more
// packets runs in passes.
constexpr uint32_t kSliceLds = 1024;

// Device-memory command words of a server launch (the leader's relay to the
// other workgroups): dcmd[seq & 1] = seq | n << 32 for every request, in
// order (a wide one before the leader serves its slice, a one-workgroup one
// after); dcmd[2] = kBurstExit << 32 | epoch: leave.  Zeroed by the host
// before every launch (seq 0 is never posted), and an exit word counts only
// with this launch's epoch.  The words are uncached device memory
// (hipDeviceMallocUncached): an sc1 poll of a cached line is served by the
// polling XCD's L2, which another XCD's store does not refresh (the cached
// word: one wide request in a suite run was not served in 2 s).
constexpr uint32_t kBurstExit = 0xffffffffu;

// A workgroup outside a request keeps its done word from lagging the seqs
// by more than kDoneLag (a word untouched for 2^31 requests would pass the
// host's serial compare for a later request it has a slice of), but stores
// only when it lags that far: every store takes the done line out of the
// host's cache, and the host reads that line at every request (31 refresh
// stores a request cost the poll loop 150-400 ns of misses a collect,
// tools/txloop_lab split).  Reading the word does not take the line.
constexpr uint32_t kDoneLag = 1u << 20;

__device__ __forceinline__ void done_refresh(BurstBox *box, uint32_t j, uint32_t seq)
{
	if (seq - sys_relaxed(&box->done[j]) > kDoneLag)
		__hip_atomic_store(&box->done[j], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint64_t relay_load(const uint64_t *p)
{
	return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void relay_store(uint64_t *p, uint64_t v)
{
	__hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void burst_server_kernel(BurstBox *box, const uint64_t *door, const uint32_t *stopw,
							   const uint8_t *req0,
							   const uint8_t *vblk, uint8_t *scratch, uint8_t *resp0,
							   uint64_t *dcmd, const void *zero, uint32_t cap,
							   uint32_t max_pkts, uint32_t per_wg, uint32_t start_seq,
							   uint32_t epoch, uint32_t opts)
{
	// cmd: 1 serve the request, 2 exit, 3 already served by an earlier launch
	__shared__ uint32_t cmd, cmd_n, cmd_seq, cmd_vram;
	__shared__ uint4 hdr_w[4];
	__shared__ uint32_t sdesc[3 * kSliceLds];
	(void)sdesc;
	__shared__ uint4 sblock[kBurstFirst / 16]; // a small request's block (the one-workgroup path)
	__shared__ uint4 szero;                    // the zero chunk of the LDS-resident body
	if (threadIdx.x == 0)
		szero = make_uint4(0, 0, 0, 0);
	const int t = threadIdx.x;
	const uint32_t j = blockIdx.x, K = gridDim.x;
	const uint32_t rslot = burst_resp_slot(max_pkts);
	uint32_t last = start_seq; // the last request seen (thread 0)
	// thread 0: requests left whose done[j] is checked first — after a relaunch
	// the (up to two) pending requests may have been served in part already
	uint32_t recheck = 2;
	for (;;) {
		if (t == 0) {
			const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
			const uint64_t idle = box->idle_ticks;
			uint32_t c = 0, n = 0;
			if (j == 0) {
				// The leader polls the host mailbox slot of the next seq.
				// Only one workgroup does: K pollers of one host line cost
				// every request ~13 us at K = 16 and ~27 us at K = 32
				// (tools/txburst dropin, one in_cksum through a server of K
				// workgroups).  The leader serves every request, so the host
				// cannot post past the one it waits for.
				const uint32_t want = burst_next(last);
				while (c == 0) {
					// relaxed: an acquire load would invalidate the caches every poll.
					// `door` is device memory the host writes through the large
					// BAR (uncached: every poll reads memory, a local read instead
					// of a round trip over the fabric), or box->req in host memory
					const uint64_t r = sys_relaxed64(&door[want & 1]);
					// the stop word beside the mailbox words: with the doorbell in
					// device memory a poll reads no host line at all (a host read
					// in the loop set its period to a fabric round trip: the
					// doorbell's gain lost, profiles/r06/)
					if (sys_relaxed(stopw))
						c = 2;
					else if ((uint32_t)r == want)
						c = 1, last = want, n = (uint32_t)(r >> 32);
					else if (__builtin_amdgcn_s_memrealtime() - t0 > idle)
						c = 2;
					else
						__builtin_amdgcn_s_sleep(4);
				}
				// relay a wide request (and the exit) to the others now; a
				// small one after it is served (it keeps their idle bound
				// from running out)
				if (K > 1 && c == 2)
					relay_store(dcmd + 2, (uint64_t)kBurstExit << 32 | epoch);
				else if (K > 1 && burst_wgs(n & ~kBurstVram, K, per_wg) > 1)
					relay_store(dcmd + (last & 1), (uint64_t)last | (uint64_t)n << 32);
			} else {
				// The others poll the leader's relay in device memory, with
				// a bound of their own (four idle periods) in case it never
				// comes.  A slot already holding a later request of its
				// parity means the host collected the one wanted, so this
				// workgroup was not part of it: step over it.
				while (c == 0) {
					const uint32_t want = burst_next(last);
					const uint64_t e = relay_load(dcmd + 2);
					const uint64_t r = relay_load(dcmd + (want & 1));
					if ((uint32_t)(e >> 32) == kBurstExit && (uint32_t)e == epoch)
						c = 2;
					else if ((uint32_t)r == want)
						c = 1, last = want, n = (uint32_t)(r >> 32);
					else if ((uint32_t)r != 0 && (int32_t)((uint32_t)r - want) > 0) {
						// not ours: on to the next seq.  Its done word
						// is kept within kDoneLag of it (done_refresh)
						last = want;
						if (!(opts & 16)) // lab bit 16: the refresh off (the regression test's control)
							done_refresh(box, j, want);
					}
					else if (__builtin_amdgcn_s_memrealtime() - t0 > 4 * idle)
						c = 2;
					else
						__builtin_amdgcn_s_sleep(2);
				}
			}
			// A relaunch after a drain re-posts the pending requests; a
			// slice the previous launch already served is not served twice
			// (an in-place store is not idempotent without ZERO_FIELDS).
			if (c == 1 && recheck) {
				--recheck;
				if ((int32_t)(sys_relaxed(&box->done[j]) - last) >= 0)
					c = 3;
			}
			cmd = c;
			cmd_n = n & ~kBurstVram;
			cmd_vram = n & kBurstVram;
			cmd_seq = last;
		}
		__syncthreads();
		if (cmd == 2)
			break;
		const uint32_t n = cmd_n, seq = cmd_seq;
		const bool vram = cmd_vram != 0 && vblk != nullptr;
		const uint32_t W = burst_wgs(n, K, per_wg);
		const uint64_t nraw = (uint64_t)(n | (vram ? kBurstVram : 0u)) << 32; // the relayed count keeps the flag
		if (j >= W || cmd == 3) {
			if (t == 0 && j == 0 && K > 1 && W == 1)
				relay_store(dcmd + (seq & 1), (uint64_t)seq | nraw);
			// a workgroup outside the request's W keeps its done word within
			// kDoneLag of the seqs (done_refresh); the host reads done[j]
			// only for j < W of the request it waits for
			if (t == 0 && cmd == 1 && !(opts & 16))
				done_refresh(box, j, seq);
			__syncthreads(); // cmd / cmd_n are rewritten by the next poll
			continue;
		}
		// lab opts bit 512: every workgroup but the leader starts its slice
		// 20 us late, so a host that took a stale done word for served would
		// read outputs not yet written (the wrap test's control)
		if ((opts & 512) && j > 0)
			for (const uint64_t d0 = __builtin_amdgcn_s_memrealtime(); __builtin_amdgcn_s_memrealtime() - d0 < 2000;)
				__builtin_amdgcn_s_sleep(8);
		const uint8_t *req = vram ? vblk + (size_t)(seq & 1) * kBurstFirst : req0 + (size_t)(seq & 1) * cap;
		uint8_t *resp = resp0 + (size_t)(seq & 1) * rslot;
		const uint4 *src = reinterpret_cast<const uint4 *>(req);
		uint4 *dst = reinterpret_cast<uint4 *>(scratch);
#if CGCK_LAB
		uint64_t lab_t0 = __builtin_amdgcn_s_memrealtime(), lab_t1 = 0, lab_t2 = 0;
		uint64_t lab_c1 = 0;
#endif
		// Host memory is cached in L2 (hipHostMallocCoherent staging too: a
		// plain read of the block served an earlier request's header), so no
		// read of it may be served from a line an earlier request left.  A
		// system-scope acquire invalidates the caches, but costs 2 us (of a
		// small request's 3 us block-read phase, tools/srvlat; an
		// agent-scope one the same): a one-workgroup request reads its first
		// block bytes with system-coherent loads (ld_sys16x2) and takes the
		// acquire only before host memory it reads with plain loads (the
		// rest of a large block, packet bytes in place); a slice of a wide
		// request takes it first.  Lab opts bit 32: before every request.
		const bool one_wg = W == 1 && !(opts & 1);
		if (!one_wg || (opts & 32))
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
		bool ok;
		// opts bits 1 / 2 (lab A/B, results then partial): no verdict stores
		// / no stores at all
		uint8_t *ver = (opts & 6) ? nullptr : resp + burst_ver_off(n);
		uint32_t *o32 = (opts & 4) ? nullptr : reinterpret_cast<uint32_t *>(resp);
		uint32_t *meta = reinterpret_cast<uint32_t *>(resp + burst_meta_off(n));
		const BurstReq &h = *reinterpret_cast<const BurstReq *>(hdr_w);
		// opts bit 0 (lab A/B): a one-workgroup request takes the slice path
		// too (header and descriptors only, packets read where they lie)
		if (one_wg) {
			// the first kBurstFirst bytes of the block in one round trip:
			// plain 16-byte loads, so every wave's read leaves as whole-line
			// requests
			static_assert(kBurstFirst == 2 * 16 * 256, "two 16-byte loads per thread");
			uint4 v0, v1;
			ld_sys16x2(src + t, src + 256 + t, v0, v1);
			if (t < 4)
				hdr_w[t] = v0;
			// A block of up to kBurstFirst bytes (a small request: every
			// drop-in call, a burst of up to ~64 small frames) stays in LDS:
			// descriptors and staged bytes are read from there (ds_read, no
			// L2 round trips); a larger one is copied into device scratch.
			sblock[t] = v0;
			sblock[256 + t] = v1;
			__syncthreads();
			ok = burst_hdr_ok(h, n, max_pkts, vram ? kBurstFirst : cap);
			// (lab opts bit 4096: the scratch copy for every block, the A/B)
			const bool in_lds = !ok || (h.bytes <= kBurstFirst && !(opts & 4096));
			const uint32_t *sd;
			if (in_lds) {
				sd = reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(sblock) + sizeof(BurstReq));
				if (ok) {
					const uint64_t limit = burst_limit(h);
					for (uint32_t i = t; i < n; i += 256)
						ok = ok && desc_inside(((lds_u32 *)sd)[3 * i], ((lds_u32 *)sd)[3 * i + 1],
								       ((lds_u32 *)sd)[3 * i + 2], limit);
				}
			} else {
				dst[t] = v0;
				dst[256 + t] = v1;
				const uint32_t chunks = (h.bytes + 15) / 16;
				// the rest of the block, 16 loads in flight per thread (64
				// KiB a round trip), plain loads after the acquire
				__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
				for (uint32_t at = kBurstFirst / 16; at < chunks; at += 16 * 256) {
					uint4 x[16];
#pragma unroll
					for (int k = 0; k < 16; ++k) {
						const uint32_t i = at + k * 256 + t;
						x[k] = i < chunks ? src[i] : make_uint4(0, 0, 0, 0);
					}
#pragma unroll
					for (int k = 0; k < 16; ++k) {
						const uint32_t i = at + k * 256 + t;
						if (i < chunks)
							dst[i] = x[k];
					}
				}
				// scratch stores visible to the workgroup (its waves share
				// one CU's L1: workgroup scope), and no line of an earlier
				// request's copy left in that L1
				__builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
				__syncthreads();
				__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
				asm volatile("buffer_inv sc0" ::: "memory");
				sd = reinterpret_cast<const uint32_t *>(scratch + sizeof(BurstReq));
				const uint64_t limit = burst_limit(h);
				for (uint32_t i = t; i < n; i += 256)
					ok = ok && desc_inside(gbl(sd)[3 * i], gbl(sd)[3 * i + 1], gbl(sd)[3 * i + 2], limit);
			}
			ok = __syncthreads_and(ok);
#if CGCK_LAB
			lab_t1 = __builtin_amdgcn_s_memrealtime();
			lab_c1 = __builtin_amdgcn_s_memtime();
#endif
			// (lab opts bit 16384: the body runs twice, lab_body timing the
			// second — warm against cold, tools/srvlat)
#if CGCK_LAB
			for (int lab_rep = 0; ok && lab_rep < ((opts & 16384) ? 2 : 1); ++lab_rep)
#endif
			if (ok) {
#if CGCK_LAB
				const uint64_t lab_b0 = __builtin_amdgcn_s_memtime();
#endif
				// staged packet bytes are read from the LDS or scratch copy;
				// packet bytes in place by the system-coherent body, or with
				// plain loads after the acquire (lab opts bit 256: always so)
				const bool sys = h.base && burst_sys_ok(h, n) && !(opts & 256);
				if (h.base && !sys)
					__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
				if (in_lds) {
					const uint8_t *base = h.base ? reinterpret_cast<const uint8_t *>(h.base)
								     : reinterpret_cast<const uint8_t *>(sblock) + h.p_off;
#if !CGCK_SERVER_SMALL_ONLY
					if (sys)
						burst_body_spec<true, true>(h, sd, n, o32, meta, ver, zero, base, opts);
					else if (h.base)
						burst_body<true>(h, sd, 0, n, o32, meta, ver, zero, base);
					else
#endif
						burst_body_spec<true, false, true>(h, sd, n, o32, meta, ver, &szero, base, opts);
				} else {
#if !CGCK_SERVER_SMALL_ONLY
					const uint8_t *base = h.base ? reinterpret_cast<const uint8_t *>(h.base) : scratch + h.p_off;
					if (sys)
						burst_body<false, true>(h, sd, 0, n, o32, meta, ver, zero, base);
					else
						burst_body<false>(h, sd, 0, n, o32, meta, ver, zero, base);
#endif
				}
#if CGCK_LAB
				if (t == 0 && j == 0)
					__hip_atomic_store(&box->lab_body, __builtin_amdgcn_s_memtime() - lab_b0, __ATOMIC_RELAXED,
							   __HIP_MEMORY_SCOPE_SYSTEM);
#endif
			}
		} else {
			// Slice [lo, hi) in passes of up to kSliceLds descriptors: the
			// header (first pass) and the pass's descriptors in one round
			// trip, as dwords (a slice starts on a 4-byte boundary), into
			// LDS; the count comes from the poll, so the slice does not
			// wait for the header.
#if CGCK_SERVER_SMALL_ONLY
			ok = false;
#else
			const uint32_t lo = (uint32_t)((uint64_t)n * j / W), hi = (uint32_t)((uint64_t)n * (j + 1) / W);
			const uint32_t *sd = reinterpret_cast<const uint32_t *>(req + sizeof(BurstReq));
			// (a device-memory block holds at most kBurstFirst bytes: no
			// descriptor read past it, whatever the mailbox word says)
			ok = n <= max_pkts && (!vram || sizeof(BurstReq) + 12ull * n <= kBurstFirst);
			for (uint32_t c0 = lo; ok && c0 < hi; c0 += kSliceLds) {
				const uint32_t c1 = hi - c0 < kSliceLds ? hi : c0 + kSliceLds;
				const uint32_t nd = 3 * (c1 - c0);
				const uint4 hv = (c0 == lo && t < 4) ? src[t] : make_uint4(0, 0, 0, 0);
				for (uint32_t i = t; i < nd; i += 4 * 256) {
					uint32_t x[4];
#pragma unroll
					for (int k = 0; k < 4; ++k)
						x[k] = i + k * 256 < nd ? gbl(sd)[3 * c0 + i + k * 256] : 0u;
#pragma unroll
					for (int k = 0; k < 4; ++k)
						if (i + k * 256 < nd)
							sdesc[i + k * 256] = x[k];
				}
				if (c0 == lo && t < 4)
					hdr_w[t] = hv;
				__syncthreads();
				ok = burst_hdr_ok(h, n, max_pkts, vram ? kBurstFirst : cap);
				if (ok) {
					const uint64_t limit = burst_limit(h);
					for (uint32_t i = t; i < c1 - c0; i += 256)
						ok = ok && desc_inside(sdesc[3 * i], sdesc[3 * i + 1], sdesc[3 * i + 2], limit);
				}
				ok = __syncthreads_and(ok);
#if CGCK_LAB
				if (c0 == lo) {
					lab_t1 = __builtin_amdgcn_s_memrealtime();
					lab_c1 = __builtin_amdgcn_s_memtime();
				}
#endif
				if (!ok)
					break;
				const uint8_t *base = h.base ? reinterpret_cast<const uint8_t *>(h.base) : req + h.p_off;
				burst_body<true, false, false, false>(h, sdesc, c0, c1, o32, meta, ver, zero, base);
				__syncthreads(); // the next pass rewrites sdesc
			}
#endif
		}
		if (!ok && t == 0) {
			__hip_atomic_store(&box->refused[seq & 1], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
			__hip_atomic_fetch_add(&box->bad_req, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
		}
#if CGCK_LAB
		__syncthreads();
		lab_t2 = __builtin_amdgcn_s_memrealtime();
		const uint64_t lab_c2 = __builtin_amdgcn_s_memtime();
#endif
		// every thread's outputs (and in-place stores) in host memory before
		// thread 0 publishes done[j].  A one-workgroup request's bodies store
		// to host memory system-coherent (WT: written through), so their own
		// completion is enough: a wait per thread, the barrier, then done[j]
		// (a system-scope release, an L2 write-back, before both cost up to
		// ~1 us a request: tools/srvlat, profiles/r05/burst/release/); a
		// wide request's slices store plainly and publish after the release.
		// Lab opts bit 2048: the release for every request.
		const bool wt = one_wg && !(opts & 2048);
		if (wt)
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		else
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
		__syncthreads();
#if CGCK_LAB
		if (t == 0 && j == 0) {
			const uint64_t lab_t3 = __builtin_amdgcn_s_memrealtime();
			__hip_atomic_store(&box->lab_t[0], lab_t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
			__hip_atomic_store(&box->lab_t[1], lab_t1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
			__hip_atomic_store(&box->lab_t[2], lab_t2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
			__hip_atomic_store(&box->lab_t[3], lab_t3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
			__hip_atomic_store(&box->lab_cyc, lab_c2 - lab_c1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
		}
#endif
		if (t == 0) {
			if (wt)
				__hip_atomic_store(&box->done[j], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
			else
				__hip_atomic_store(&box->done[j], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
			if (j == 0 && K > 1 && W == 1)
				relay_store(dcmd + (seq & 1), (uint64_t)seq | nraw);
		}
	}
	if (t == 0)
		__hip_atomic_store(&box->alive[j], (uint8_t)0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_burst_server(BurstBox *box, const uint64_t *door, const uint32_t *stopw, const uint8_t *req,
			       const uint8_t *vblk, uint8_t *scratch, uint8_t *resp, uint64_t *dcmd, const void *zero,
			       uint32_t cap, uint32_t max_pkts, uint32_t wgs, uint32_t per_wg, uint32_t start_seq,
			       uint32_t epoch, uint32_t opts, hipStream_t st)
{
	hipError_t e = hipMemsetAsync(dcmd, 0, 3 * sizeof(uint64_t), st);
	if (e != hipSuccess)
		return e;
	hipLaunchKernelGGL(burst_server_kernel, dim3(wgs), dim3(256), 0, st, box, door, stopw, req, vblk, scratch, resp,
			   dcmd, zero, cap, max_pkts, per_wg, start_seq, epoch, opts);
	return hipGetLastError();
}

template <int G, int S, int U, bool DESC>
static hipError_t launch_t(const KParams &p, int max_blocks, bool nt, hipStream_t st)
{
	constexpr uint64_t PPB = (256 / G) * U;
	uint64_t want = (p.n + PPB - 1) / PPB;
	int blocks = (int)(want < (uint64_t)max_blocks ? want : (uint64_t)max_blocks);
	if (blocks < 1)
		blocks = 1;
	if (nt) {
		CGCK_NOTE_KERNEL("cksum_kernel<%d, %d, %d, %s, true>", G, S, U, tf(DESC));
		hipLaunchKernelGGL((cksum_kernel<G, S, U, DESC, true>), dim3(blocks), dim3(256), 0, st, p);
	} else {
		CGCK_NOTE_KERNEL("cksum_kernel<%d, %d, %d, %s, false>", G, S, U, tf(DESC));
		hipLaunchKernelGGL((cksum_kernel<G, S, U, DESC, false>), dim3(blocks), dim3(256), 0, st, p);
	}
	return hipGetLastError();
}

hipError_t launch_group(const KParams &p, uint32_t max_len, int num_cus, bool nt, hipStream_t st)
{
	// 48 blocks per CU: 80.4 % vs 78.5-78.9 % at 24 and 78.2 % at 16 on one box
	// (tools/bpc_sweep.sh): shorter contiguous block ranges
	static const int bpc = [] { // $CGCK_GRP_BPC: blocks per CU (A/B runs)
		const char *e = CGCK_ENV("CGCK_GRP_BPC");
		return e && atoi(e) > 0 ? atoi(e) : 48;
	}();
	const int max_blocks = num_cus * bpc;
	const bool d = p.desc != nullptr;
	if (max_len <= 80) // <= 6 chunks at any alignment: two steps of 4 lanes
		return d ? launch_t<4, 2, 4, true>(p, max_blocks, nt, st)
			 : launch_t<4, 2, 4, false>(p, max_blocks, nt, st);
	if (max_len <= 256)
		return d ? launch_t<16, 2, 2, true>(p, max_blocks, nt, st)
			 : launch_t<16, 2, 2, false>(p, max_blocks, nt, st);
	if (max_len <= 768) // 576 B (IMIX's middle class): 48 chunks per group, two packets per group step
		return d ? launch_t<16, 3, 2, true>(p, max_blocks, nt, st)
			 : launch_t<16, 3, 2, false>(p, max_blocks, nt, st);
	if (max_len <= 1600)
		return d ? launch_t<16, 6, 1, true>(p, max_blocks, nt, st)
			 : launch_t<16, 6, 1, false>(p, max_blocks, nt, st);
	return d ? launch_t<64, 4, 1, true>(p, max_blocks, nt, st)
		 : launch_t<64, 4, 1, false>(p, max_blocks, nt, st);
}

} // namespace cgck
