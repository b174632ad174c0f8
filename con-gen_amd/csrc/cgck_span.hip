// cgck_span.hip — descriptor batches whose frames are packed back to back
// (cgck_set_desc_layout(CGCK_LAYOUT_PACKED); the IMIX batch of
// cgck_synth_imix is laid out this way).
//
// The lane and slot kernels read each packet on its own, so a wave's load
// instruction touches 64 separate places (lane-strided) whatever the packet
// sizes.  Here a wave instead streams the contiguous byte span that holds a
// tile of up to 64 consecutive packets, lane-consecutive 16-byte chunks, one
// fully coalesced kilobyte per load instruction — the read shape of the
// 1500 B group kernel, for any mix of lengths.
//
// Packets are separated with prefix sums, not per-packet reductions.  In the
// one's-complement arithmetic of subr.c:137-156 a sum over bytes [A, E) of
// the span is P(E) - P(A) (mod 65535), P = the running word sum from the
// span's 16-byte aligned start (the ABSOLUTE word frame of the other
// kernels, so odd starts are byte-swapped in result()).  The stream pass
// keeps C(j) = P(16 j) for every chunk j of the span in LDS: one DPP scan
// per load instruction.  A packet then needs C at its first and end chunks
// plus the bytes of those two chunks before its boundaries; its lane reads
// them back (L2 hits, the wave streamed them a moment ago) together with the
// header chunks for the header facts of header()/result() (cgck_lane.hip:
// IP header, pseudo-header, stored fields, verdicts).  Any packet inside the
// span is correct — gaps, order and overlaps only cost efficiency — so a
// tile whose span would be mostly gaps (a ring of 2048-byte slots with small
// frames) takes a plain lane-per-packet pass instead.
//
// No in-place stores (CGCK_STORE): a packet's result reads chunks its
// neighbours also read, and a neighbour's field store would race with them;
// the dispatcher keeps STORE batches on the other families.
#include "cgck_lane.h"

#include <stdlib.h>

namespace cgck {

#ifndef CGCK_SPAN_MAXC // (variant builds for A/B runs override these two)
#define CGCK_SPAN_MAXC 1536
#define CGCK_SPAN_S 24
#endif
constexpr int kSpanMaxC = CGCK_SPAN_MAXC; // chunks per tile span (24 KiB; 64 IMIX packets take ~22.7 KiB)
constexpr int kSpanS = CGCK_SPAN_S;       // chunk loads in flight per lane: a whole tile span in one step
// Outputs leave in windows of kSpanStage packets per wave (LDS staging, one
// burst of nontemporal stores per window): a per-tile store would put its
// write acknowledgement in front of the next tile's loads (in-order vmcnt).
constexpr int kSpanStage = 512;

// one lane's packet without the span: its own chunks, lane-strided
__device__ __forceinline__ uint32_t lane_total(const uint4 *c0, int nch, int q, int len, const void *zero)
{
	uint32_t tot = 0;
	for (int t = 0; __any(t < nch); t += 4) {
		uint4 w[4];
#pragma unroll
		for (int i = 0; i < 4; ++i)
			w[i] = ldc<false>(c0, t + i, nch, zero);
		uint32_t s = 0;
#pragma unroll
		for (int i = 0; i < 4; ++i)
			s = t + i < nch ? sum4(w[i], s) : s;
		tot = fold16(tot) + fold16(s);
	}
	if (nch > 0) {
		const uint4 first = ldc<false>(c0, 0, nch, zero), last = ldc<false>(c0, nch - 1, nch, zero);
		const int e = q + len - 16 * (nch - 1);
		uint32_t corr = fold16(lead_sum(first, q, false)) + fold16(trail_sum(last, e, false));
		tot = ocsub(fold16(tot), fold16(corr));
	}
	return fold16(tot);
}

// max over the wave, on every lane's result via lane 63 (row shifts, then the
// row broadcasts of lanes 15 and 31)
__device__ __forceinline__ uint32_t wave_max_dpp(uint32_t x)
{
	x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false)); // row_shr:1
	x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false)); // row_shr:2
	x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false)); // row_shr:4
	x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false)); // row_shr:8
	x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false)); // row_bcast:15
	x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false)); // row_bcast:31
	return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

template <bool NT>
__global__ __launch_bounds__(256) void span_kernel(KParams p)
{
	__shared__ uint16_t cpre[4][kSpanMaxC + 2];
	__shared__ uint32_t so[4][kSpanStage];
	__shared__ uint8_t sv[4][kSpanStage];
	const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
	const uint64_t nwaves = (uint64_t)gridDim.x * 4;
	const uint64_t wid = (uint64_t)blockIdx.x * 4 + wv;
	const uint64_t per = (p.n + nwaves - 1) / nwaves;
	const uint64_t r0 = wid * per;
	const uint64_t r1 = r0 + per < p.n ? r0 + per : p.n;
	const bool raw = p.flags & CGCK_RAW;
	uint16_t *C = cpre[wv];
	uint64_t sb = r0; // first packet of the open output window
	auto flush = [&](uint64_t e) { // wave-uniform
		__builtin_amdgcn_wave_barrier();
		asm volatile("" ::: "memory");
		for (int i = l; sb + i < e; i += 64) {
			if (p.out)
				__builtin_nontemporal_store(so[wv][i], gbl(p.out) + sb + i);
			if (p.verdict)
				gbl(p.verdict)[sb + i] = sv[wv][i];
		}
		__builtin_amdgcn_wave_barrier();
		asm volatile("" ::: "memory");
		sb = e;
	};
	DescW dn = load_desc<true>(p, r0 + l, r1);
	for (uint64_t cur = r0; cur < r1;) {
		const Pkt pk = decode<true>(p, cur + l, r1, dn);
		const int len = (int)pk.len, q = (int)(pk.a0 & 15), nch = nchunks(pk.a0, pk.len);
		const uint4 *c0 = reinterpret_cast<const uint4 *>(pk.a0 & ~(uint64_t)15);
		// the tile: the leading packets whose bytes lie within kSpanMaxC chunks
		// of lane 0's chunk (lane 0 always holds a packet: cur < r1)
		const uint64_t R0 = (((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(pk.a0 >> 32), 0) << 32) |
				     (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)pk.a0, 0)) & ~(uint64_t)15;
		const uint64_t E = pk.a0 + pk.len;
		const bool fits = pk.ok && pk.a0 >= R0 && E - R0 <= (uint64_t)kSpanMaxC * 16;
		const uint64_t fm = __ballot(fits);
		const int m = ~fm ? __builtin_ctzll(~fm) : 64;
		const bool in = l < m;
		// span end (max) and packet bytes (sum) over the tile: DPP, no LDS trips
		const uint32_t rel = wave_max_dpp(in ? (uint32_t)(E - R0) : 0u);
		const uint32_t bytes = (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_dpp(in ? (uint32_t)len : 0u), 63);
		const int RC = (int)((rel + 15) >> 4); // chunks of the span
		const bool span = m > 0 && (uint32_t)RC * 16 <= 2 * bytes + 1024;
		const int adv = span ? m : (int)(r1 - cur < 64 ? r1 - cur : 64);
		// the next tile's descriptors load while this one streams
		dn = load_desc<true>(p, cur + adv + l, r1);
		uint64_t k = cur + l;
		Res r;
		bool act;
		if (span) {
			// Each packet's header chunks and end-boundary chunk load first,
			// lane by lane, then the stream of the whole span: the stream's
			// loads of those lines hit in L2 (or merge with the misses in
			// flight), and nothing is read back after the stream — a re-read
			// would miss L2 at this occupancy (tens of KiB per wave in flight).
			const uint4 *R = reinterpret_cast<const uint4 *>(R0);
			act = in;
			const uint32_t A = (uint32_t)(pk.a0 - R0), Eo = A + (uint32_t)len;
			const int cs = in ? (int)(A >> 4) : 0, ce = in ? (int)(Eo >> 4) : 0;
			uint4 v[4];
#pragma unroll
			for (int i = 0; i < 4; ++i)
				v[i] = ldc<false>(c0, i, in ? nch : 0, p.zero);
			const uint4 vce = ldc<false>(R, in ? ce : 0, in ? RC : 0, p.zero); // chunk of the end boundary
			// ---- stream pass: C(j) for every chunk of the span ----
			// Buffer loads through a descriptor of exactly the span: one
			// 32-bit lane offset for every load (the step in the scalar
			// offset), and chunks past the span read as zero by the range
			// check instead of a per-load clamp.
			const uint32_t blo = __builtin_amdgcn_readfirstlane((uint32_t)R0),
				       bhi = __builtin_amdgcn_readfirstlane((uint32_t)(R0 >> 32));
			const int nbytes = __builtin_amdgcn_readfirstlane(RC * 16);
			const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
				reinterpret_cast<void *>(((uint64_t)bhi << 32) | blo), 0, nbytes, 0x00020000);
			uint32_t carry = 0;
			for (int j0 = 0; j0 < RC; j0 += 64 * kSpanS) {
				uint4 w[kSpanS];
#pragma unroll
				for (int i = 0; i < kSpanS; ++i) {
					const u32x4_t x = __builtin_amdgcn_raw_buffer_load_b128(rsrc, l * 16, (j0 + 64 * i) * 16,
												 NT ? 2 : 0);
					w[i] = make_uint4(x[0], x[1], x[2], x[3]);
				}
#pragma unroll
				for (int i = 0; i < kSpanS; ++i) {
					const int j = j0 + 64 * i + l;
					const uint32_t cs_ = sum4(w[i], 0);
					const uint32_t incl = wave_scan_dpp(cs_);
					if (j < RC)
						C[j] = (uint16_t)fold16(carry + incl - cs_);
					carry = fold16(carry + (uint32_t)__builtin_amdgcn_readlane((int)incl, 63));
				}
			}
			if (l == 0)
				C[RC] = (uint16_t)carry;
			__builtin_amdgcn_wave_barrier();
			asm volatile("" ::: "memory");
			// ---- per packet: boundaries from C ----
			// (v[0] is chunk cs whenever the packet has bytes; an empty one sums to 0)
			uint32_t T = ocsub((uint32_t)C[ce], (uint32_t)C[cs]);
			T = fold16(T + fold16(lead_sum(vce, (int)(Eo & 15), false)));
			T = len ? ocsub(T, fold16(lead_sum(v[0], q, false))) : 0u;
			Hdr h{};
			if (!raw)
				h = header<4, false>(v, c0, in ? nch : 0, q, len, p.flags, act);
			r = result(p, pk.a0, len, T, h);
		} else {
			// ---- lane per packet: a sparse tile ----
			act = pk.ok;
			uint4 v[4];
#pragma unroll
			for (int i = 0; i < 4; ++i)
				v[i] = ldc<false>(c0, i, act ? nch : 0, p.zero);
			const uint32_t T = lane_total(c0, act ? nch : 0, q, len, p.zero);
			Hdr h{};
			if (!raw)
				h = header<4, false>(v, c0, act ? nch : 0, q, len, p.flags, act);
			r = result(p, pk.a0, len, T, h);
		}
		if (cur + adv > sb + kSpanStage)
			flush(cur);
		if (act) {
			so[wv][k - sb] = r.out;
			sv[wv][k - sb] = (uint8_t)r.verdict;
		}
		__builtin_amdgcn_wave_barrier(); // C is rewritten by the next tile
		asm volatile("" ::: "memory");
		cur += adv;
	}
	if (r0 < r1)
		flush(r1);
}

bool span_ok(const KParams &p)
{
	return p.desc && !(p.flags & (CGCK_STORE | kFlagNoLenCheck | kFlagL4Auto));
}

hipError_t launch_span(const KParams &p, int num_cus, bool nt, hipStream_t st)
{
	// Exactly the resident blocks: every wave owns 1/(grid x 4) of the
	// batch, so a grid larger than what fits at once (registers, LDS) would
	// run its last blocks alone.  $CGCK_SPAN_BPC overrides (A/B runs).
	static const int bpc_env = [] {
		const char *e = CGCK_ENV("CGCK_SPAN_BPC");
		return e ? atoi(e) : 0;
	}();
	static const int fit[2] = {
		[] {
			int b = 0;
			return hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, span_kernel<false>, 256, 0) == hipSuccess && b > 0 ? b : 2;
		}(),
		[] {
			int b = 0;
			return hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, span_kernel<true>, 256, 0) == hipSuccess && b > 0 ? b : 2;
		}(),
	};
	const int bpc = bpc_env > 0 ? bpc_env : fit[nt];
	const uint64_t want = (p.n + 4 * 64 - 1) / (4 * 64), mb = (uint64_t)num_cus * bpc;
	const dim3 g((unsigned)(want < mb ? want : mb));
	if (nt) {
		CGCK_NOTE_KERNEL("span_kernel<true>");
		hipLaunchKernelGGL(span_kernel<true>, g, dim3(256), 0, st, p);
	} else {
		CGCK_NOTE_KERNEL("span_kernel<false>");
		hipLaunchKernelGGL(span_kernel<false>, g, dim3(256), 0, st, p);
	}
	return hipGetLastError();
}

} // namespace cgck
