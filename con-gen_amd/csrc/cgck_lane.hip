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
#include "cgck_lane.h"

#include <stdlib.h>

namespace cgck {

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
#if CGCK_LAB // A/B-only: software-pipelined lpp (lpa replaced it)
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

#endif // CGCK_LAB

// --------------------------------------------------------------------------
// Lane per packet, aligned fixed-length strided batches (the 64 B config)
// --------------------------------------------------------------------------
//
// Strided batch, base/stride/l3_off all multiples of 16 and one ip_len in
// [20, 64]: every packet is nch = ceil(len/16) whole chunks from a 16-byte
// boundary, the same for every lane.  Chunk loads are unconditional (index
// clamped to the last chunk, idle lanes to packet n-1), so no load sits in
// a branch and every wait is a counted vmcnt.  Two packet groups per lane
// are in flight (explicit A/B registers, no loop-carried copies): the
// chunks of group i+1 are issued before group i is reduced and its output
// stored, so each output store trails the next group's loads (vmcnt retires
// in order on gfx9).
struct Quad {
	uint4 c[4];
};

template <bool NT>
__device__ __forceinline__ void lpa_load(const KParams &p, uint64_t k, bool live, int nch, Quad &q)
{
	k = k < p.n ? k : p.n - 1;
	// past the block's last group: a zero line of the context, one of 64 by
	// block, instead of re-reading packet bytes that have left the L2
	const uint4 *c0 = live ? reinterpret_cast<const uint4 *>(p.base + k * p.stride + p.l3_off)
			       : reinterpret_cast<const uint4 *>((const uint8_t *)p.zero + (blockIdx.x & 63) * 64);
#pragma unroll
	for (int i = 0; i < 4; ++i)
		q.c[i] = ld<NT>(c0 + (i < nch ? i : nch - 1));
}

// Reduce packet k's quad and store its u32 output.  The store carries the
// nontemporal policy: +3 points of HBM peak in the slower of the two states a
// process lands in, +1.5 in the faster (tools/ab_lib.sh; the same policy on
// the group, slot and hash kernels' stores lost up to 13 points).  (A staged
// form — four results per lane leaving as one 16-byte store after an LDS
// transpose — measured 66.7 % vs 69.5 % of HBM peak on one box.)
template <bool NT, bool STAGE = false>
__device__ __forceinline__ void lpa_reduce(const KParams &p, uint64_t k, int len, int nch, const Quad &q,
					   uint32_t *so = nullptr)
{
	const bool ok = k < p.n;
	// Fast path (wave-uniform): ip_cksum + tcp_cksum only, whole chunks, and
	// every packet of the wave with ip_hl = 5 — the 64 B config.  IP header =
	// dwords 0..4, pseudo src/dst = dwords 3..4, ip_p = byte 9; the same
	// arithmetic as result() with no field, verdict or store work.
	if (p.flags == (CGCK_IP | CGCK_L4) && (len & 15) == 0 && !__any(ok && (q.c[0].x & 15u) != 5u)) {
		uint32_t T = 0;
#pragma unroll
		for (int i = 0; i < 4; ++i)
			if (i < nch)
				T = sum4(q.c[i], T);
		const uint32_t IPs = fold16(hsum(q.c[1].x, sum4(q.c[0], 0)));
		const uint32_t PS = fold16(hsum(q.c[1].x, hsum(q.c[0].w, 0)));
		const uint32_t proto = (q.c[0].z >> 8) & 0xffu;
		uint32_t L = ocsub(fold16(T), IPs);
		L = fold16(L + PS + (proto << 8) + bswap16((uint32_t)(len - 20)));
		if (ok) {
			const uint32_t out = finish(IPs) | (finish(L) << 16);
			if (STAGE) {
				*so = out;
			} else if (p.out) {
				uint32_t *o = p.out + k;
				asm volatile("global_store_dword %0, %1, off nt" ::"v"(o), "v"(out) : "memory");
			}
			if (p.verdict)
				gbl(p.verdict)[k] = 0;
		}
		return;
	}
	// chunks 4, 5 are zero: len <= 64 puts every header and L4-field dword
	// header() may read below dword 16, so it never loads more
	uint4 v[6];
	v[4] = v[5] = make_uint4(0, 0, 0, 0);
#pragma unroll
	for (int i = 0; i < 4; ++i) {
		// wave-uniform: chunks past the packet drop out, the last one keeps
		// its first len - 16 i bytes
		const int r1 = i < nch - 1 ? 16 : (i == nch - 1 ? len - 16 * i : 0);
		v[i] = make_uint4(q.c[i].x & dmask(0, 0, 0, r1), q.c[i].y & dmask(0, 1, 0, r1),
				  q.c[i].z & dmask(0, 2, 0, r1), q.c[i].w & dmask(0, 3, 0, r1));
	}
	uint32_t tot = 0;
#pragma unroll
	for (int i = 0; i < 4; ++i)
		tot = sum4(v[i], tot);
	const uint64_t a0 = reinterpret_cast<uint64_t>(p.base) + (ok ? k : 0) * p.stride + p.l3_off;
	Hdr h{};
	if (!(p.flags & CGCK_RAW))
		h = header<6, NT>(v, reinterpret_cast<const uint4 *>(a0), nch, 0, len, p.flags, ok);
	if (ok) {
		const Res r = result(p, a0, len, fold16(tot), h);
		if (p.out) {
			// The u32 output through inline asm: the compiler then does not
			// hold the next group's address/data registers (which it tends to
			// allocate onto this store's data VGPR) behind a vmcnt(0) for the
			// store.  Every vmcnt the compiler computes stays conservative: the
			// hidden store only makes in-order waits include it.
			if (STAGE) {
				*so = r.out;
			} else {
				uint32_t *o = p.out + k;
				asm volatile("global_store_dword %0, %1, off nt" ::"v"(o), "v"(r.out) : "memory");
			}
		}
		if (p.verdict)
			gbl(p.verdict)[k] = (uint8_t)r.verdict;
	}
}

template <bool NT, int DEPTH>
__global__ __launch_bounds__(256) void lpa_kernel(KParams p)
{
	const int len = (int)p.ip_len, nch = (len + 15) >> 4;
	const uint64_t NI = (p.n + 255) / 256, S = gridDim.x;
	uint64_t it = blockIdx.x;
	if (it >= NI)
		return;
	// DEPTH packet groups per lane in a register ring: the load of group
	// d + DEPTH - 1 is issued before group d is reduced.  Loads are never
	// skipped (past the end they read a zero line), so the loop has no load
	// under a branch and every wait is a counted vmcnt.
	Quad Q[DEPTH];
#pragma unroll
	for (int d = 0; d < DEPTH - 1; ++d)
		lpa_load<NT>(p, (it + d * S) * 256 + threadIdx.x, it + d * S < NI, nch, Q[d]);
	for (;;) {
#pragma unroll
		for (int d = 0; d < DEPTH; ++d) {
			const uint64_t ahead = it + (uint64_t)(d + DEPTH - 1) * S;
			lpa_load<NT>(p, ahead * 256 + threadIdx.x, ahead < NI, nch, Q[(d + DEPTH - 1) % DEPTH]);
			lpa_reduce<NT>(p, (it + d * S) * 256 + threadIdx.x, len, nch, Q[d]);
			if (it + (uint64_t)(d + 1) * S >= NI)
				return;
		}
		it += (uint64_t)DEPTH * S;
	}
}

// --------------------------------------------------------------------------
// Lane per packet fed by LDS-DMA (lpd: the 64 B config's default)
// --------------------------------------------------------------------------
//
// lpa's per-lane loads touch 64 lines per instruction.  Here each step of 64
// packets (63 * stride + len <= 4 KiB) moves as four contiguous 1 KiB
// global_load_lds_dwordx4 instructions into a ring of D LDS slots of its
// wave, and lane L reads packet L's chunks from LDS and reduces them with
// lpa_reduce (the same arithmetic).  Steps come in chunks of C, and chunks
// are grid-interleaved (wave b takes chunks b, b + G, ...), so the grid sweeps
// one window of the batch: the DMA sweep alone then reads 89-99 % of 8 TB/s
// (a contiguous range per wave: 78-89 %).  The output stores were the cost
// left (92 % with the reduce but no stores, 74 % with a u32 store per packet),
// so a chunk's outputs are staged in LDS and leave as one contiguous
// C * 256-byte run of 16-byte stores (sc1 policy).  In one process on one
// buffer (tools/sweep.py, profiles/r02/lpd/): C = 32, D = 2, 8 waves per CU,
// sc1 stores 80.6 % against lpa's 71.8 %; C = 16 75.2 %, nt stores 78.8 %,
// default-policy stores 73.1 %, D = 3 or 10 waves per CU lose (LDS occupancy
// below the grid: a tail of non-resident waves).
//
// Counted vmcnt: per step 4 DMA; a chunk flush adds C / 4 stores, so the wait
// for step j leaves the D - 1 later steps' DMA and, right after a flush, the
// flush's stores in flight.
template <int D, int C, int SP>
__global__ __launch_bounds__(64) void lpd_kernel(KParams p)
{
	extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
	const int lane = threadIdx.x;
	const int len = (int)p.ip_len, nch = (len + 15) >> 4;
	const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem);
	uint32_t *so = reinterpret_cast<uint32_t *>(smem + D * 4096); // C > 1: a chunk's outputs
	const uint8_t *zero = (const uint8_t *)p.zero + (blockIdx.x & 63) * 64;
	const uint64_t base = reinterpret_cast<uint64_t>(p.base) + p.l3_off;
	const uint64_t last_chunk = (base + (p.n - 1) * p.stride + len - 1) & ~(uint64_t)15;
	// Chunks of C steps of 64 packets, grid-interleaved (wave b takes chunks
	// b, b + G, ...): the grid sweeps one window of the batch, so reads and
	// output writes stay within few DRAM pages chip-wide.  C > 1: a chunk's
	// outputs are staged in LDS and leave as one contiguous C * 256-byte run.
	const uint64_t NS = (p.n + 63) / 64, NC = (NS + C - 1) / C, G = gridDim.x, b = blockIdx.x;
	if (b >= NC)
		return;
	const uint64_t nsteps = (NC - b + G - 1) / G * C;
	auto gstep = [&](uint64_t j) { return (b + (j / C) * G) * C + j % C; };
	// bytes a step covers: lanes past them (stride < 64) read the zero line
	const uint32_t span = (uint32_t)(63 * p.stride) + (uint32_t)len;
	auto issue = [&](uint64_t j) { // step j of this wave into slot j % D
		const uint64_t gs = gstep(j);
		const uint64_t a = base + gs * 64 * p.stride;
		const uint32_t slot = lds0 + (uint32_t)(j % D) * 4096;
#pragma unroll
		for (int i = 0; i < 4; ++i) {
			const uint32_t at = 1024 * i + 16 * lane;
			const uint64_t src = a + at;
			glds16_nt(j < nsteps && gs < NS && at < span && src <= last_chunk ? reinterpret_cast<const void *>(src)
											  : zero,
				  slot + 1024 * i);
		}
	};
#pragma unroll
	for (int d = 0; d < D - 1; ++d)
		issue(d);
	const int o = lane * (int)p.stride; // packet L's byte offset in a slot
	constexpr bool stage = C > 1; // lpd_ok guarantees an output array
	// SP >= 3 (lab A/B): a full chunk's outputs are read from the staging into
	// registers at the chunk's end and stored right AFTER the next step's DMA
	// issue (as lpw does), so the two following waits leave them in flight
	// (two steps to complete instead of one); store policy SP - 3.
	constexpr bool DEFER = SP >= 3 && C > 1;
	constexpr int policy = SP % 3 == 0 ? kNt : SP % 3 == 1 ? kDefaultPolicy : kSc1;
	u32x4_t held[DEFER ? C / 4 : 1];
	bool pend = false;
	uint64_t pfirst = 0;
	for (uint64_t j = 0; j < nsteps; ++j) {
		issue(j + D - 1);
		if (DEFER && pend) {
			const __amdgpu_buffer_rsrc_t rs = out_rsrc(p.out + pfirst, C * 256);
#pragma unroll
			for (int i = 0; i < (DEFER ? C / 4 : 0); ++i)
				bstore16<policy>(rs, 16 * (i * 64 + lane), held[i]);
			pend = false;
		}
		// Wait for step j's DMA.  Issued after it: the DMA of the D - 1 later
		// steps, plus the output stores of the steps since (C == 1: one per
		// step once the ring is full; C > 1: C / 4 of the last chunk flush,
		// when that flush came after step j's DMA).
		if (C == 1) {
			if (j + 1 < (uint64_t)D || !p.out)
				asm volatile("s_waitcnt vmcnt(%0)" ::"i"(4 * (D - 1)) : "memory");
			else
				asm volatile("s_waitcnt vmcnt(%0)" ::"i"(5 * (D - 1)) : "memory");
		} else {
			if (stage && j >= (uint64_t)C && (j % C) <= (uint64_t)(DEFER ? D - 1 : D - 2))
				asm volatile("s_waitcnt vmcnt(%0)" ::"i"(4 * (D - 1) + C / 4) : "memory");
			else
				asm volatile("s_waitcnt vmcnt(%0)" ::"i"(4 * (D - 1)) : "memory");
		}
		__builtin_amdgcn_s_barrier();
		const uint8_t *sl = smem + (uint32_t)(j % D) * 4096;
		Quad q;
#pragma unroll
		for (int i = 0; i < 4; ++i)
			q.c[i] = *reinterpret_cast<const uint4 *>(sl + o + 16 * (i < nch ? i : nch - 1));
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // the slot is refilled next step
		const uint64_t k = gstep(j) * 64 + lane;
		if (stage)
			lpa_reduce<false, true>(p, k, len, nch, q, so + (j % C) * 64 + lane);
		else
			lpa_reduce<false>(p, k, len, nch, q);
		if (stage && (j + 1) % C == 0 && p.contig != 2) { // contig 2: lab $CGCK_LPD_SINK, no flush
			// flush the chunk: C / 4 coalesced 16-byte stores per lane
			const uint64_t first = (b + (j / C) * G) * C * 64;
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
			if (DEFER && first + C * 64 <= p.n && j + 1 < nsteps) {
				const u32x4_t *s4 = reinterpret_cast<const u32x4_t *>(so);
#pragma unroll
				for (int i = 0; i < (DEFER ? C / 4 : 0); ++i)
					held[i] = s4[i * 64 + lane];
				asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // read before the next reduce restages
				pend = true;
				pfirst = first;
			} else if (first + C * 64 <= p.n) {
				const uint4 *s4 = reinterpret_cast<const uint4 *>(so);
				const __amdgpu_buffer_rsrc_t rs = out_rsrc(p.out + first, C * 256);
#pragma unroll
				for (int i = 0; i < C / 4; ++i) {
					const uint4 w = s4[i * 64 + lane];
					bstore16<policy>(rs, 16 * (i * 64 + lane), u32x4_t{w.x, w.y, w.z, w.w});
				}
			} else {
				// the batch's last, partial chunk: per-packet stores, then drain
				for (int i = lane; i < C * 64; i += 64)
					if (first + i < p.n)
						gbl(p.out)[first + i] = so[i];
				asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			}
		}
	}
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

#if CGCK_LAB
// Loader/consumer form (A/B; lost: 62-72 %): the output store sits in the
// consumers' vmcnt only.
// Wave 0 of a 256-thread workgroup only moves bytes (a phase = 3 steps of 64
// packets, 12 KiB, into a ring of P phases); waves 1..3 each reduce one step
// per phase from LDS and store its outputs.  Per phase: the loader waits
// (counted vmcnt) for phase ph, all four waves pass barrier ph, the loader
// refills the slots of phase ph - 1 (which the consumers finished,
// lgkmcnt(0), before that barrier) with phase ph + P - 1.
template <int P>
__global__ __launch_bounds__(256) void lpd_lc_kernel(KParams p)
{
	extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
	const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const int lane = threadIdx.x & 63;
	const int len = (int)p.ip_len, nch = (len + 15) >> 4;
	const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem);
	const uint8_t *zero = (const uint8_t *)p.zero + (blockIdx.x & 63) * 64;
	const uint64_t base = reinterpret_cast<uint64_t>(p.base) + p.l3_off;
	const uint64_t last_chunk = (base + (p.n - 1) * p.stride + len - 1) & ~(uint64_t)15;
	// phases of 192 packets, grid-interleaved (workgroup b takes phases b,
	// b + G, ...), as in the per-wave form
	const uint64_t NP = (p.n + 191) / 192, G = gridDim.x, b = blockIdx.x;
	if (b >= NP)
		return; // uniform across the workgroup
	const uint64_t nph = (NP - b + G - 1) / G;
	if (wave == 0) {
		auto issue = [&](uint64_t ph) {
			const uint32_t grp = lds0 + (uint32_t)(ph % P) * 3 * 4096;
#pragma unroll
			for (int c = 0; c < 3; ++c) {
				const uint64_t first = (b + ph * G) * 192 + 64 * c;
				const uint64_t a = base + first * p.stride;
#pragma unroll
				for (int i = 0; i < 4; ++i) {
					const uint64_t src = a + 1024 * i + 16 * lane;
					glds16_nt(ph < nph && first < p.n && src <= last_chunk ? reinterpret_cast<const void *>(src) : zero,
						  grp + c * 4096 + 1024 * i);
				}
			}
		};
#pragma unroll
		for (int d = 0; d < P - 1; ++d)
			issue(d);
		for (uint64_t ph = 0; ph < nph; ++ph) {
			// phase ph landed: phases ph + 1 .. ph + P - 2 may stay in flight
			asm volatile("s_waitcnt vmcnt(%0)" ::"i"((P - 2) * 12) : "memory");
			__builtin_amdgcn_s_barrier();
			issue(ph + P - 1);
		}
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	} else {
		const int c = wave - 1;
		const int o = lane * (int)p.stride;
		for (uint64_t ph = 0; ph < nph; ++ph) {
			__builtin_amdgcn_s_barrier();
			const uint64_t first = (b + ph * G) * 192 + 64 * c;
			if (first < p.n) {
				const uint8_t *sl = smem + ((uint32_t)(ph % P) * 3 + c) * 4096;
				Quad q;
#pragma unroll
				for (int i = 0; i < 4; ++i)
					q.c[i] = *reinterpret_cast<const uint4 *>(sl + o + 16 * (i < nch ? i : nch - 1));
				asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
				lpa_reduce<false>(p, first + lane, len, nch, q);
			}
			// this phase's slots are refilled after the next barrier
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
		}
	}
}

// lpd with a writer wave (A/B): wave 0 of a 128-thread workgroup is
// lpd_kernel's DMA ring and reduce without any global store; at the end of a
// chunk it hands the staged outputs to wave 1 across a barrier, and wave 1
// reads them into registers (before the next step's barrier, so wave 0 may
// refill the staging) and stores them as 16-byte sc1 runs.  The stores then
// count only in the writer's vmcnt, not in front of wave 0's DMA waits.
template <int D, int C>
__global__ __launch_bounds__(128) void lpdw_kernel(KParams p)
{
	extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
	const int lane = threadIdx.x & 63;
	const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const int len = (int)p.ip_len, nch = (len + 15) >> 4;
	const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem);
	uint32_t *so = reinterpret_cast<uint32_t *>(smem + D * 4096); // a chunk's outputs
	const uint8_t *zero = (const uint8_t *)p.zero + (blockIdx.x & 63) * 64;
	const uint64_t base = reinterpret_cast<uint64_t>(p.base) + p.l3_off;
	const uint64_t last_chunk = (base + (p.n - 1) * p.stride + len - 1) & ~(uint64_t)15;
	const uint64_t NS = (p.n + 63) / 64, NC = (NS + C - 1) / C, G = gridDim.x, b = blockIdx.x;
	if (b >= NC)
		return;
	const uint64_t nsteps = (NC - b + G - 1) / G * C;
	if (wave == 1) {
		for (uint64_t j = 0; j < nsteps; ++j) {
			wg_barrier();
			if ((j + 1) % C != 0)
				continue;
			wg_barrier(); // chunk j / C staged
			const uint64_t first = (b + (j / C) * G) * C * 64;
			if (first + C * 64 <= p.n) {
				u32x4_t v[C / 4];
				const uint4 *s4 = reinterpret_cast<const uint4 *>(so);
#pragma unroll
				for (int i = 0; i < C / 4; ++i) {
					const uint4 w = s4[i * 64 + lane];
					v[i] = u32x4_t{w.x, w.y, w.z, w.w};
				}
				asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // staging free before the next barrier
				const __amdgpu_buffer_rsrc_t rs = out_rsrc(p.out + first, C * 256);
#pragma unroll
				for (int i = 0; i < C / 4; ++i)
					bstore16<kSc1>(rs, 16 * (i * 64 + lane), v[i]);
			} else {
				for (int i = lane; i < C * 64; i += 64)
					if (first + i < p.n)
						gbl(p.out)[first + i] = so[i];
				asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
			}
		}
		return;
	}
	auto gstep = [&](uint64_t j) { return (b + (j / C) * G) * C + j % C; };
	const uint32_t span = (uint32_t)(63 * p.stride) + (uint32_t)len;
	auto issue = [&](uint64_t j) {
		const uint64_t gs = gstep(j);
		const uint64_t a = base + gs * 64 * p.stride;
		const uint32_t slot = lds0 + (uint32_t)(j % D) * 4096;
#pragma unroll
		for (int i = 0; i < 4; ++i) {
			const uint32_t at = 1024 * i + 16 * lane;
			const uint64_t src = a + at;
			glds16_nt(j < nsteps && gs < NS && at < span && src <= last_chunk ? reinterpret_cast<const void *>(src)
											  : zero,
				  slot + 1024 * i);
		}
	};
#pragma unroll
	for (int d = 0; d < D - 1; ++d)
		issue(d);
	const int o = lane * (int)p.stride;
	for (uint64_t j = 0; j < nsteps; ++j) {
		issue(j + D - 1);
		asm volatile("s_waitcnt vmcnt(%0)" ::"i"(4 * (D - 1)) : "memory");
		wg_barrier();
		const uint8_t *sl = smem + (uint32_t)(j % D) * 4096;
		Quad q;
#pragma unroll
		for (int i = 0; i < 4; ++i)
			q.c[i] = *reinterpret_cast<const uint4 *>(sl + o + 16 * (i < nch ? i : nch - 1));
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // the slot is refilled next step
		const uint64_t k = gstep(j) * 64 + lane;
		lpa_reduce<false, true>(p, k, len, nch, q, so + (j % C) * 64 + lane);
		if ((j + 1) % C == 0) {
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // the chunk's outputs are in LDS
			wg_barrier();                      // hand them to the writer
		}
	}
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

#endif // CGCK_LAB

bool lpd_ok(const KParams &p)
{
	// an output array, 16-byte aligned: a chunk's outputs leave as 16-byte stores
	return !p.desc && !p.verdict && !p.bad && !(p.flags & CGCK_STORE) && p.out &&
	       (reinterpret_cast<uintptr_t>(p.out) & 15) == 0 && p.ip_len >= 20 && p.ip_len <= 64 &&
	       p.stride <= 64 && p.stride * 63 + p.ip_len <= 4096 &&
	       ((reinterpret_cast<uintptr_t>(p.base) | p.stride | p.l3_off) & 15) == 0;
}

hipError_t launch_lpd(const KParams &p, int num_cus, hipStream_t st)
{
	static const int wpc = [] { // $CGCK_LPD_WPC: waves per CU
		const char *e = CGCK_ENV("CGCK_LPD_WPC");
		return e && atoi(e) > 0 ? atoi(e) : 8;
	}();
	const uint64_t want = (p.n + 64 * 16 - 1) / (64 * 16); // >= 16 steps per wave
	const uint64_t cap = (uint64_t)num_cus * wpc;
	const dim3 g((unsigned)(want < cap ? (want ? want : 1) : cap));
#if CGCK_LAB
	static const int depth = [] { // $CGCK_LPD_D: ring slots 2..4
		const char *e = CGCK_ENV("CGCK_LPD_D");
		const int d = e ? atoi(e) : 0;
		return d >= 2 && d <= 4 ? d : 2;
	}();
	static const int lc = [] { // $CGCK_LPD_LC: ring phases of the loader/consumer form (0: per-wave form)
		const char *e = CGCK_ENV("CGCK_LPD_LC");
		const int v = e ? atoi(e) : 0;
		return v >= 2 && v <= 5 ? v : 0;
	}();
	if (lc) {
		static const int wgpc = [] { // $CGCK_LPD_WGPC: workgroups per CU
			const char *e = CGCK_ENV("CGCK_LPD_WGPC");
			return e && atoi(e) > 0 ? atoi(e) : 3;
		}();
		const uint64_t want_lc = (p.n + 192 * 16 - 1) / (192 * 16); // >= 16 phases per workgroup
		const uint64_t cap_lc = (uint64_t)num_cus * wgpc;
		const dim3 glc((unsigned)(want_lc < cap_lc ? (want_lc ? want_lc : 1) : cap_lc));
#define CGCK_LPDLC(PP)                                                                           \
	do {                                                                                     \
		CGCK_NOTE_KERNEL("lpd_lc_kernel<%d>", PP);                                       \
		hipLaunchKernelGGL((lpd_lc_kernel<PP>), glc, dim3(256), (PP) * 3 * 4096, st, p); \
	} while (0)
		switch (lc) {
		case 2: CGCK_LPDLC(2); break;
		case 4: CGCK_LPDLC(4); break;
		case 5: CGCK_LPDLC(5); break;
		default: CGCK_LPDLC(3); break;
		}
#undef CGCK_LPDLC
		return hipGetLastError();
	}
	static const int wr = [] { // $CGCK_LPD_W: lpdw_kernel (writer wave), steps per chunk 16 | 32
		const char *e = CGCK_ENV("CGCK_LPD_W");
		return e ? atoi(e) : 0;
	}();
	if (wr == 16 || wr == 32) {
		if (wr == 16) {
			CGCK_NOTE_KERNEL("lpdw_kernel<%d, 16>", 2);
			hipLaunchKernelGGL((lpdw_kernel<2, 16>), g, dim3(128), 2 * 4096 + 16 * 256, st, p);
		} else {
			CGCK_NOTE_KERNEL("lpdw_kernel<%d, 32>", 2);
			hipLaunchKernelGGL((lpdw_kernel<2, 32>), g, dim3(128), 2 * 4096 + 32 * 256, st, p);
		}
		return hipGetLastError();
	}
	static const bool sink = CGCK_ENV("CGCK_LPD_SINK") != nullptr; // measure without output stores
	KParams q = p;
	if (sink)
		q.contig = 2;
	static const int chunk = [] { // $CGCK_LPD_C: steps per output chunk (1, 4, 8, 16, 32, 64)
		const char *e = CGCK_ENV("CGCK_LPD_C");
		const int c = e ? atoi(e) : 32;
		return c == 1 || c == 4 || c == 8 || c == 16 || c == 64 ? c : 32;
	}();
	static const int sp = [] { // $CGCK_LPD_SP: flush store policy 0 nt, 1 default, 2 sc1
		const char *e = CGCK_ENV("CGCK_LPD_SP");
		const int v = e ? atoi(e) : 2;
		return v >= 0 && v <= 5 ? v : 2; // 3..5: the same, stored after the next step's issue
	}();
#define CGCK_LPD_S(DD, CC, SS)                                                                   \
	do {                                                                                     \
		CGCK_NOTE_KERNEL("lpd_kernel<%d, %d, %d>", DD, CC, SS);                          \
		hipLaunchKernelGGL((lpd_kernel<DD, CC, SS>), g, dim3(64), (DD) * 4096 + (CC) * 256, st, q); \
	} while (0)
#define CGCK_LPD(DD, CC)                                                                         \
	do {                                                                                     \
		if (sp == 1)                                                                     \
			CGCK_LPD_S(DD, CC, 1);                                                   \
		else if (sp == 0)                                                                \
			CGCK_LPD_S(DD, CC, 0);                                                   \
		else                                                                             \
			CGCK_LPD_S(DD, CC, 2);                                                   \
	} while (0)
#define CGCK_LPD_D(DD)                                                                           \
	do {                                                                                     \
		if (chunk == 1)                                                                  \
			CGCK_LPD(DD, 1);                                                         \
		else if (chunk == 4)                                                             \
			CGCK_LPD(DD, 4);                                                         \
		else if (chunk == 8)                                                             \
			CGCK_LPD(DD, 8);                                                         \
		else if (chunk == 16)                                                            \
			CGCK_LPD(DD, 16);                                                        \
		else if (chunk == 64)                                                            \
			CGCK_LPD(DD, 64);                                                        \
		else                                                                             \
			CGCK_LPD(DD, 32);                                                        \
	} while (0)
	if (sp == 5 && depth == 2 && chunk == 32) { // the deferred flush, sc1 (lab A/B)
		CGCK_LPD_S(2, 32, 5);
		return hipGetLastError();
	}
	switch (depth) {
	case 3: CGCK_LPD_D(3); break;
	case 4: CGCK_LPD_D(4); break;
	default: CGCK_LPD_D(2); break;
	}
#undef CGCK_LPD_D
#undef CGCK_LPD
#undef CGCK_LPD_S
#else
	CGCK_NOTE_KERNEL("lpd_kernel<2, 32, 2>");
	hipLaunchKernelGGL((lpd_kernel<2, 32, 2>), g, dim3(64), 2 * 4096 + 32 * 256, st, p);
#endif
	return hipGetLastError();
}

hipError_t launch_lpa(const KParams &p, int num_cus, bool nt, hipStream_t st)
{
	// One block per CU (one wave per SIMD) with four packet groups per lane in
	// flight: 68.8-69.1 % of HBM peak vs 66.2-66.4 % for two groups at 3 blocks
	// per CU and 67.9-68.7 % for three groups (tools/lpa_depth.sh, one box).
	// The per-packet reduce is short, so fewer waves with deeper register
	// rings keep more bytes in flight per instruction issued.
	static const int bpc = [] { // $CGCK_LPA_BPC: blocks per CU (A/B runs)
		const char *e = CGCK_ENV("CGCK_LPA_BPC");
		return e && atoi(e) > 0 ? atoi(e) : 1;
	}();
	static const int depth = [] { // $CGCK_LPA_DEPTH: packet groups per lane in flight, 2..4
		const char *e = CGCK_ENV("CGCK_LPA_DEPTH");
		const int d = e ? atoi(e) : 0;
		return d >= 2 && d <= 4 ? d : 4;
	}();
	uint64_t want = (p.n + 255) / 256, mb = (uint64_t)num_cus * bpc;
	const dim3 g((unsigned)(want < mb ? want : mb));
#define CGCK_LPA(D)                                                                            \
	do {                                                                                   \
		if (nt) {                                                                      \
			CGCK_NOTE_KERNEL("lpa_kernel<true, %d>", D);                           \
			hipLaunchKernelGGL((lpa_kernel<true, D>), g, dim3(256), 0, st, p);      \
		} else {                                                                       \
			CGCK_NOTE_KERNEL("lpa_kernel<false, %d>", D);                          \
			hipLaunchKernelGGL((lpa_kernel<false, D>), g, dim3(256), 0, st, p);     \
		}                                                                              \
	} while (0)
	if (depth == 4)
		CGCK_LPA(4);
	else if (depth == 3)
		CGCK_LPA(3);
	else
		CGCK_LPA(2);
#undef CGCK_LPA
	return hipGetLastError();
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

#if CGCK_LAB // A/B-only: the first lane-per-slot design (slot2 replaced it)
template <bool DESC, bool NT>
__global__ __launch_bounds__(256) void slot_kernel(KParams p)
{
	__shared__ uint32_t mark[4][64];
	__shared__ uint32_t so[4][kWaveStage];
	__shared__ uint8_t sv[4][kWaveStage];
	const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63; // wave-uniform (SGPR)
	const bool raw = p.flags & CGCK_RAW;
	const uint64_t nwaves = (uint64_t)gridDim.x * 4;
	const uint64_t wid = (uint64_t)blockIdx.x * 4 + wv;
	const uint64_t per = (p.n + nwaves - 1) / nwaves;
	const uint64_t r0 = wid * per;
	const uint64_t r1 = r0 + per < p.n ? r0 + per : p.n;
	WaveStage ws{so[wv], sv[wv], r0};

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
			wave_stage_reserve(p, ws, cur, 1);
			if (l == 0)
				wave_stage_put(ws, cur, result(p, a0, len, fold16(acc), h));
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
			w[i] = ldc<NT>(c0, 8 * s + i, nch, p.zero);
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
		wave_stage_reserve(p, ws, cur, m);
		if (head)
			wave_stage_put(ws, cur + owner, result(p, a0, len, fold16(r), h));
		cur += m;
	}
	if (r0 < r1)
		wave_stage_flush(p, ws, r1);
}

#endif // CGCK_LAB

// --------------------------------------------------------------------------
// Lane per 128-byte slot, software-pipelined two deep
// --------------------------------------------------------------------------
//
// Same slot mapping as slot_kernel, but a wave keeps TWO iterations of chunk
// loads in flight: while iteration i is reduced, the chunks of i+1 are
// loading and the descriptors of i+2 too.  In-order vmcnt retirement shapes
// the issue order of each phase:
//
//   map(i+1) [waits only for desc(i+1), issued before chunks(i)]
//   issue desc(i+2); issue chunks(i+1)
//   reduce(i) [waits for chunks(i): desc(i+2) + chunks(i+1) stay in flight]
//
// The A/B buffers are explicit (the loop body is unrolled twice) so no
// register holding an in-flight load is ever copied — a copy would force a
// vmcnt(0) at the back edge.  Every load is branch-free (clamped to the
// packet's chunks or the context's zero chunk) so vmcnt counting stays exact.

// One iteration's lane -> (packet, slot) mapping.
struct SMap {
	uint64_t a0;   // owner packet's IPv4 header (jumbo: lane 0's packet)
	int len, nch;  // owner packet
	int s;         // slot index inside the owner packet
	int st, ns;    // owner's first slot (lane) and slot count
	int owner;     // owner's packet index relative to the iteration
	int m;         // packets placed this iteration (0: jumbo or empty)
	bool act;      // lane holds a slot
};

template <bool DESC>
__device__ __forceinline__ SMap smap(const KParams &p, uint64_t cur, uint64_t r1, const DescW &d,
				     uint32_t (&mark)[64])
{
	const int l = threadIdx.x & 63;
	const Pkt pk = decode<DESC>(p, cur + l, r1, d);
	const int nch_l = nchunks(pk.a0, pk.len);
	const uint32_t ns = pk.ok ? (uint32_t)max(1, (nch_l + 7) >> 3) : 0u;
	const uint32_t P = wave_scan_dpp(ns);
	const uint64_t fit = __ballot(pk.ok && P <= 64);
	SMap M;
	M.m = __popcll(fit);
	const int T = M.m ? (int)__builtin_amdgcn_readlane(P, M.m - 1) : 0; // slots in use
	mark[l] = 0;
	__builtin_amdgcn_wave_barrier();
	asm volatile("" ::: "memory");
	if (l < M.m)
		mark[P - ns] = 1;
	__builtin_amdgcn_wave_barrier();
	asm volatile("" ::: "memory");
	const uint64_t heads = __ballot(mark[l] != 0 && l < T);
	const uint64_t le = l == 63 ? ~0ull : ((2ull << l) - 1);
	const uint64_t below = heads & le, above = heads & ~le;
	M.act = l < T;
	M.owner = below ? __popcll(below) - 1 : 0;
	M.st = below ? 63 - __clzll(below) : 0;
	M.ns = (above ? __ffsll((long long)above) - 1 : T) - M.st;
	M.s = l - M.st;
	M.a0 = shfl64(pk.a0, M.owner);
	M.len = __shfl((int)pk.len, M.owner, 64);
	M.nch = nchunks(M.a0, (uint32_t)M.len);
	return M;
}

template <bool NT>
__device__ __forceinline__ void slot_issue(const KParams &p, const SMap &M, uint4 (&w)[8])
{
	// Idle lanes (past the slots in use) clamp into the last placed packet's
	// final chunk, a line its own tail lane reads anyway: pointing them all
	// at the context's one zero chunk made every wave of the grid hit the
	// same address (one L2 channel).  Their chunks are excluded from sums.
	const uint4 *c0 = reinterpret_cast<const uint4 *>(M.a0 & ~(uint64_t)15);
#pragma unroll
	for (int i = 0; i < 8; ++i)
		w[i] = ldc<NT>(c0, 8 * M.s + i, M.nch, p.zero);
}

template <bool NT>
__device__ __forceinline__ void slot_reduce(const KParams &p, uint64_t cur, const SMap &M, uint4 (&w)[8],
					    WaveStage &ws)
{
	const int l = threadIdx.x & 63;
	const bool raw = p.flags & CGCK_RAW;
	const uint64_t a0 = M.a0;
	const int len = M.len, nch = M.nch, s = M.s;
	const int q = (int)(a0 & 15);
	const uint4 *c0 = reinterpret_cast<const uint4 *>(a0 & ~(uint64_t)15);
	// All of w[] counts as consumed here, on every path: a chunk whose use
	// sits in a skippable branch (or the jumbo path, which ignores w[]) would
	// leave its load "maybe pending" and degrade later waits to vmcnt(0).
#pragma unroll
	for (int i = 0; i < 8; ++i)
		asm volatile("" ::"v"(w[i].x), "v"(w[i].y), "v"(w[i].z), "v"(w[i].w));
	if (M.m == 0) {
		// jumbo packet (> 64 slots): windows of 64 slots, whole-wave sums
		const int nsj = (nch + 7) >> 3;
		uint32_t acc = 0;
		Hdr h{};
		for (int wbase = 0; wbase < nsj; wbase += 64) {
			const int sj = wbase + l;
			// the window reuses w[] (dead here) with clamped, branch-free loads
			uint4 (&v)[8] = w;
#pragma unroll
			for (int i = 0; i < 8; ++i)
				v[i] = ldc<NT>(c0, 8 * sj + i, nch, p.zero);
			uint32_t r = 0;
#pragma unroll
			for (int i = 0; i < 8; ++i)
				r = 8 * sj + i < nch ? sum4(v[i], r) : r;
			if (wbase == 0 && !raw)
				h = header<8, NT>(v, c0, nch, q, len, p.flags, l == 0);
			const int j = (nch - 1) - 8 * sj;
			const int e = q + len - 16 * (nch - 1);
			uint32_t corr = 0;
			if (sj == 0 && q != 0)
				corr += lead_sum(v[0], q, false);
			if (j >= 0 && j < 8 && e != 16)
				corr += trail_sum(pick8(v, j), e, false);
			r = fold16(r) + (0xffffu - fold16(corr));
			acc = fold16(acc) + fold16(gsum<64>(r));
		}
		wave_stage_reserve(p, ws, cur, 1);
		if (l == 0)
			wave_stage_put(ws, cur, result(p, a0, len, fold16(acc), h));
		// drain this rare path completely so the wait state merged after it
		// holds no "maybe pending" loads (they would cost a vmcnt(0) later)
		__builtin_amdgcn_s_waitcnt(0);
		return;
	}
	const bool act = M.act;
	uint32_t r = 0;
#pragma unroll
	for (int i = 0; i < 8; ++i)
		r = act && 8 * s + i < nch ? sum4(w[i], r) : r;
	const bool head = act && s == 0;
	Hdr h{};
	if (!raw)
		h = header<8, NT>(w, c0, nch, q, len, p.flags, head);
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
		nso |= __any(act && ((M.ns >> b) & 1)) ? (1u << b) : 0u;
	const int send = M.st + M.ns;
#pragma unroll
	for (int d = 1; d < 64; d <<= 1) {
		if ((uint32_t)d >= nso)
			break;
		const uint32_t y = __shfl_down(r, d, 64);
		if (l + d < send)
			r += y;
	}
	wave_stage_reserve(p, ws, cur, M.m);
	if (head)
		wave_stage_put(ws, cur + M.owner, result(p, a0, len, fold16(r), h));
}

#if !CGCK_LAB || !defined(CGCK_SLOT2_CHUNK) // compile-time A/B knob of the lab build only
#undef CGCK_SLOT2_CHUNK
#define CGCK_SLOT2_CHUNK 0
#endif
template <bool DESC, bool NT>
__global__ __launch_bounds__(256) void slot2_kernel(KParams p)
{
	__shared__ uint32_t mark[4][64];
	__shared__ uint32_t so[4][kWaveStage];
	__shared__ uint8_t sv[4][kWaveStage];
	const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63; // wave-uniform (SGPR)
	const uint64_t nwaves = (uint64_t)gridDim.x * 4;
	const uint64_t wid = (uint64_t)blockIdx.x * 4 + wv;
#if CGCK_SLOT2_CHUNK
	// chunks of CGCK_SLOT2_CHUNK packets, grid-interleaved (A/B builds)
	for (uint64_t ck = wid; ck * CGCK_SLOT2_CHUNK < p.n; ck += nwaves) {
	const uint64_t r0 = ck * CGCK_SLOT2_CHUNK;
	const uint64_t r1 = r0 + CGCK_SLOT2_CHUNK < p.n ? r0 + CGCK_SLOT2_CHUNK : p.n;
#else
	const uint64_t per = (p.n + nwaves - 1) / nwaves;
	const uint64_t r0 = wid * per;
	const uint64_t r1 = r0 + per < p.n ? r0 + per : p.n;
	if (r0 >= r1)
		return;
#endif
	WaveStage ws{so[wv], sv[wv], r0};

	// prologue: map A, desc of B, chunks of A
	uint64_t curA = r0;
	SMap mA = smap<DESC>(p, curA, r1, load_desc<DESC>(p, curA + l, r1), mark[wv]);
	uint64_t curB = curA + (mA.m ? mA.m : 1);
	DescW dB = load_desc<DESC>(p, curB + l, r1);
	uint4 wA[8], wB[8];
	slot_issue<NT>(p, mA, wA);
	for (;;) {
		// phase A: map B, prefetch desc C, issue chunks B, reduce A
		const SMap mB = smap<DESC>(p, curB, r1, dB, mark[wv]);
		const uint64_t curC = curB + (mB.m ? mB.m : 1);
		const DescW dC = load_desc<DESC>(p, curC + l, r1);
		slot_issue<NT>(p, mB, wB);
		slot_reduce<NT>(p, curA, mA, wA, ws);
		if (curB >= r1)
			break;
		// phase B: map C, prefetch desc D, issue chunks C (into A), reduce B
		const SMap mC = smap<DESC>(p, curC, r1, dC, mark[wv]);
		const uint64_t curD = curC + (mC.m ? mC.m : 1);
		dB = load_desc<DESC>(p, curD + l, r1);
		slot_issue<NT>(p, mC, wA);
		slot_reduce<NT>(p, curB, mB, wB, ws);
		if (curC >= r1)
			break;
		curA = curC;
		mA = mC;
		curB = curD;
	}
	wave_stage_flush(p, ws, r1);
#if CGCK_SLOT2_CHUNK
	}
#endif
}

#if CGCK_LAB
// --------------------------------------------------------------------------
// Lane per 128-byte slot fed by LDS-DMA (slotd: IMIX, A/B against slot2)
// --------------------------------------------------------------------------
//
// slot2's register loads sit at the register-load read ceiling (the probe on
// the same buffer: 71.6-73.1 %), while grid-interleaved LDS-DMA reads run near
// the HBM peak (lpd_kernel).  Same slot map as slot2 (smap); each step's slots
// are moved by 8 DMA instructions into an 8 KiB LDS slot of a 2-deep ring:
// instruction i, lane l moves chunk (l & 7) of slot 8 i + (l >> 3), so an
// instruction reads up to 1 KiB contiguous of one packet and slot s lands at
// +128 s.  Lane s then reads its 8 chunks back from LDS and reduces them with
// slot_reduce.  One wave per workgroup; chunks of kSlotdChunk descriptors are
// grid-interleaved.  Descriptor loads are the compiler's (its vmcnt waits for
// them also cover the DMA issued before, which only makes them stricter); the
// wait for a step's DMA is explicit: only the next step's 8 DMA stay in flight.
constexpr int kSlotdChunk = 2048;

template <bool NT>
__device__ __forceinline__ void slotd_issue(const KParams &p, const SMap &M, bool live, uint32_t lds_slot,
					    const uint8_t *zero)
{
	const int l = threadIdx.x & 63;
	// per slot (lane sigma of M): its first chunk and the chunks it holds
	const uint64_t cb = (M.a0 & ~(uint64_t)15) + 128 * (uint64_t)M.s;
	int rem = M.nch - 8 * M.s;
	rem = !live || !M.act || M.m == 0 ? 0 : rem < 0 ? 0 : rem > 8 ? 8 : rem;
	const uint32_t cb_lo = (uint32_t)cb, cb_hi = (uint32_t)(cb >> 32);
	const int c = l & 7;
#pragma unroll
	for (int i = 0; i < 8; ++i) {
		const int sg = 8 * i + (l >> 3);
		const uint32_t lo = __shfl(cb_lo, sg, 64), hi = __shfl(cb_hi, sg, 64);
		const int r = __shfl(rem, sg, 64);
		const uint64_t src = ((uint64_t)hi << 32 | lo) + 16 * (uint64_t)(c < r ? c : r - 1);
		glds16_nt(r > 0 ? reinterpret_cast<const void *>(src) : zero, lds_slot + 1024 * i);
	}
}

template <bool DESC>
__global__ __launch_bounds__(64) void slotd_kernel(KParams p)
{
	extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
	uint32_t *mark = reinterpret_cast<uint32_t *>(smem + 2 * 8192);
	uint32_t *so = mark + 64;
	uint8_t *sv = reinterpret_cast<uint8_t *>(so + kWaveStage);
	const int l = threadIdx.x & 63;
	const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem);
	const uint8_t *zero = (const uint8_t *)p.zero + (blockIdx.x & 63) * 64;
	for (uint64_t ck = blockIdx.x; ck * kSlotdChunk < p.n; ck += gridDim.x) {
		const uint64_t r0 = ck * kSlotdChunk;
		const uint64_t r1 = r0 + kSlotdChunk < p.n ? r0 + kSlotdChunk : p.n;
		WaveStage ws{so, sv, r0};
		uint64_t cur = r0;
		SMap M = smap<DESC>(p, cur, r1, load_desc<DESC>(p, cur + l, r1), *reinterpret_cast<uint32_t(*)[64]>(mark));
		slotd_issue<false>(p, M, true, lds0, zero);
		uint64_t curN = cur + (M.m ? M.m : 1);
		DescW dN = load_desc<DESC>(p, curN + l, r1);
		for (uint32_t j = 0;; ++j) {
			const SMap MN = smap<DESC>(p, curN, r1, dN, *reinterpret_cast<uint32_t(*)[64]>(mark));
			const uint64_t curNN = curN + (MN.m ? MN.m : 1);
			const DescW dNN = load_desc<DESC>(p, curNN + l, r1);
			slotd_issue<false>(p, MN, curN < r1, lds0 + ((j + 1) & 1) * 8192, zero);
			// step j's DMA (and everything before it) has landed: only the
			// next step's 8 DMA may stay in flight
			asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
			__builtin_amdgcn_s_barrier();
			const uint4 *sl = reinterpret_cast<const uint4 *>(smem + (j & 1) * 8192) + 8 * l;
			uint4 w[8];
#pragma unroll
			for (int i = 0; i < 8; ++i)
				w[i] = sl[i];
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // the slot is refilled next step
			slot_reduce<false>(p, cur, M, w, ws);
			if (curN >= r1)
				break;
			cur = curN;
			M = MN;
			curN = curNN;
			dN = dNN;
		}
		wave_stage_flush(p, ws, r1);
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // the last (zero) DMA landed before the ring is reused
	}
}

hipError_t launch_slotd(const KParams &p, int num_cus, hipStream_t st)
{
	static const int wpc = [] { // $CGCK_SLOTD_WPC: waves per CU
		const char *e = CGCK_ENV("CGCK_SLOTD_WPC");
		return e && atoi(e) > 0 ? atoi(e) : 6;
	}();
	const uint64_t want = (p.n + kSlotdChunk - 1) / kSlotdChunk;
	const uint64_t cap = (uint64_t)num_cus * wpc;
	const dim3 g((unsigned)(want < cap ? (want ? want : 1) : cap));
	const size_t lds = 2 * 8192 + 64 * 4 + kWaveStage * 4 + kWaveStage;
	if (p.desc) {
		CGCK_NOTE_KERNEL("slotd_kernel<true>");
		hipLaunchKernelGGL((slotd_kernel<true>), g, dim3(64), lds, st, p);
	} else {
		CGCK_NOTE_KERNEL("slotd_kernel<false>");
		hipLaunchKernelGGL((slotd_kernel<false>), g, dim3(64), lds, st, p);
	}
	return hipGetLastError();
}
#endif // CGCK_LAB

// --------------------------------------------------------------------------
// Lane per packet over DMA'd windows of the batch's own span (lpw: packed
// descriptor batches, the IMIX config under CGCK_LAYOUT_PACKED)
// --------------------------------------------------------------------------
//
// A step is 64 consecutive descriptors, one per lane.  When their chunk
// ranges chain (each packet starts at or after the starts before it and at
// or before the furthest end so far: frames back to back, as a burst copied
// into one buffer or the IMIX set), every chunk of the step's span [S, E)
// belongs to one of them.  The span is then streamed with contiguous DMA in
// windows of kLpwWin chunks through a 2-deep LDS ring; per window, a lane per
// chunk sums every chunk (conflict-free 16-byte LDS reads) and prefix-sums
// them in lane order, and a lane per packet takes its chunks' sum as a
// difference of two prefixes, minus the bytes of its edge chunks outside it;
// its header chunks are gathered in registers from whichever windows hold
// them and read once per step.  No slot map: a step's descriptors do not
// depend on the previous step, and they travel by DMA with the data (768 B,
// one instruction, into a 2-deep descriptor ring) two steps ahead, so no wait
// in the loop is on a compiler-tracked load; every round issues kLpwDma + 1
// DMA instructions (zero lines where there is nothing to move), so the waits
// are counted.  Steps that do not chain are computed from global memory by
// the same lanes (exact, slow): the layout hint says which batches chain.
// In one process on the 16M IMIX batch (tools/sweep.py,
// profiles/r02/dma/lpw/): 69.9 % of 8 TB/s against slot2's 63.8 %; windows of
// 7 / 9 / 10+ DMA instructions, fewer waves per CU, or the lane-per-packet walk
// of each window (21-23 %) lose.
#if !CGCK_LAB || !defined(CGCK_LPW_DMA) // compile-time A/B knobs of the lab build only
#undef CGCK_LPW_DMA
#define CGCK_LPW_DMA 8
#endif
// 0: instruction i moves chunks [64 i, 64 i + 64) of the window (1 KiB
// contiguous); 1: lane l moves chunks [8 l, 8 l + 8) over the 8 instructions,
// so its own run lands in conflict-free LDS places (A/B builds)
#if !CGCK_LAB || !defined(CGCK_LPW_SLOTMAJOR)
#undef CGCK_LPW_SLOTMAJOR
#define CGCK_LPW_SLOTMAJOR 0
#endif
// 1: the window's prefix with a lane per pair of chunks (4 wave scans a
// window), 0: a lane per chunk (8) — the A/B builds' knob
#if !CGCK_LAB || !defined(CGCK_LPW_PAIR)
#undef CGCK_LPW_PAIR
#define CGCK_LPW_PAIR 1
#endif
// LDS index (in 16-byte units) of window chunk idx
__device__ __forceinline__ int lpw_at(int idx)
{
#if CGCK_LPW_SLOTMAJOR
	return ((idx & 7) << 6) | (idx >> 3);
#else
	return idx;
#endif
}
constexpr int kLpwDma = CGCK_LPW_DMA;            // data DMA instructions per window
constexpr int kLpwWin = kLpwDma * 64;            // chunks a window owns (no overlap: a header
						 // split over two windows is gathered from both)
constexpr int kLpwSlot = kLpwDma * 1024;         // bytes per ring slot

struct LpwStep {
	uint64_t a0;
	int len, q, nch, e;
	bool ok;
	uint64_t cs, ce; // the lane's packet in window coordinates: absolute chunks (chained) or list positions
	uint64_t dl;     // gathered: (a0 >> 4) - cs, the chunk address of list position x is dl + x
	uint64_t S, E;   // wave: span
	uint32_t nwin;   // wave: windows (0: computed from global memory)
	bool gather;     // wave: the windows are the packets' chunk runs concatenated in lane order
};

template <bool DESC>
__device__ __forceinline__ LpwStep lpw_step(const KParams &p, uint64_t first, const DescW &d)
{
	const int l = threadIdx.x & 63;
	const Pkt pk = decode<DESC>(p, first + l, p.n, d);
	LpwStep s;
	s.a0 = pk.a0;
	s.len = (int)pk.len;
	s.ok = pk.ok;
	s.q = (int)(pk.a0 & 15);
	s.nch = nchunks(pk.a0, pk.len);
	s.e = s.q + s.len - 16 * (s.nch - 1);
	s.cs = pk.a0 >> 4;
	s.ce = s.cs + (uint64_t)s.nch;
	// Over the non-empty packets in lane order: running maxima of the starts
	// and of the ends (inclusive DPP scans of 32-bit offsets from the first
	// non-empty packet, then shifted by one lane).  The step chains when every
	// start is >= the starts before it and <= the furthest end before it: then
	// [S, E) is exactly the union of the packets' chunks.
	const bool ne = s.ok && s.nch > 0;
	const uint64_t nonempty = __ballot(ne);
	const int f = nonempty ? __ffsll((long long)nonempty) - 1 : 0; // first non-empty lane
	// the wave's values (base, span, windows) by readlane: scalar, so the
	// window loop and the round bookkeeping (pre, pend, sage) stay uniform
	// branches instead of exec-masked ones
	const uint64_t base = readlane64(s.cs, f);
	const uint64_t ds = s.cs - base, de = s.ce - base;
	const bool far = ne && (s.cs < base || de > 0x7fffffffull); // before the first, or too far for 32 bits
	const uint32_t rs = ne && !far ? (uint32_t)ds : 0u, re = ne && !far ? (uint32_t)de : 0u;
	const uint32_t mS = wave_max_scan_dpp(rs), mE = wave_max_scan_dpp(re);
	const uint32_t prev_s = (uint32_t)__shfl_up((int)mS, 1, 64), prev_e = (uint32_t)__shfl_up((int)mE, 1, 64);
	const bool brk = far || (ne && l > f && (rs < prev_s || rs > prev_e));
	s.S = nonempty ? base : 0;
	s.E = nonempty ? base + (uint64_t)__builtin_amdgcn_readlane(mE, 63) : 0;
	s.dl = 0;
	s.gather = false;
	const uint64_t span = s.E - s.S;
	if (!__any(brk) && span <= 16 * kLpwWin) {
		s.nwin = span ? (uint32_t)((span + kLpwWin - 1) / kLpwWin) : 1u; // (empty packets: one window, nothing moved)
	} else {
		// Not back to back (ring slots, gaps, reordered frames): the windows
		// walk the list of the packets' chunk runs concatenated in lane order,
		// packet p at list positions [P_p, P_p + nch_p) (an exclusive scan of
		// the chunk counts), gathered by the same DMA (lpw_issue).  The
		// per-window work is unchanged in list coordinates.
		const uint32_t nc = ne ? (uint32_t)s.nch : 0u;
		const uint32_t incl = wave_scan_dpp(nc);
		const uint32_t T = (uint32_t)__builtin_amdgcn_readlane(incl, 63);
		s.cs = incl - nc;
		s.ce = incl;
		s.dl = (pk.a0 >> 4) - s.cs;
		s.S = 0;
		s.E = T;
		s.gather = true;
		s.nwin = T > 16 * kLpwWin ? 0u : T ? (T + kLpwWin - 1) / kLpwWin : 1u;
	}
	s.nwin = __builtin_amdgcn_readfirstlane(s.nwin);
	return s;
}

// One round: window t of step s (live) or zero lines, plus the descriptors
// of step dstep (when dlive) into the descriptor slot.  A gathered step
// (gather) maps each list position of the window to its packet's chunk: the
// packets starting in the window mark their position in an owner table built
// in the target slot itself (free until this round's DMA lands; every row's
// address is computed before the first DMA is issued), a max-scan per row of 64
// positions fills the table forward, the row's carry is the last packet that
// started before it (a ballot), and the chunk address is that packet's dl
// (staged next to the table) plus the position.
template <bool DESC>
__device__ __forceinline__ void lpw_issue(const KParams &p, uint64_t wb, uint64_t E, bool live, bool gather,
					  uint64_t cs, uint64_t ce, uint64_t dl, uint8_t *slot, uint32_t lds_slot,
					  uint64_t dfirst, bool dlive, uint32_t lds_dslot, const uint8_t *zero)
{
	// window [wb, wb + 512) of a span ending at E (values, not a step
	// reference: selecting between two steps' structs put them in scratch)
	const int l = threadIdx.x & 63;
	const uint32_t base = __builtin_amdgcn_readfirstlane(lds_slot); // wave-uniform: M0
	if (gather && live) {
		uint32_t *own = reinterpret_cast<uint32_t *>(slot);       // kLpwWin entries: owner lane + 1, 0 none
		uint64_t *dls = reinterpret_cast<uint64_t *>(slot + 4 * kLpwWin); // 64 lanes' dl
		// one element type for the table, and memory clobbers between the
		// phases: the reads must not move above the zeroing or the marks (the
		// slot holds the last window's packet bytes until it is cleared)
#pragma unroll
		for (int r = 0; r < kLpwDma; ++r)
			own[64 * r + l] = 0u;
		asm volatile("" ::: "memory");
		const bool ne = ce > cs;
		if (ne && cs >= wb && cs < wb + kLpwWin)
			own[cs - wb] = (uint32_t)l + 1;
		dls[l] = dl;
		asm volatile("" ::: "memory");
		// every row's address first: row i's DMA lands on bytes [1024 i, 1024 i
		// + 1024) of the slot, over the table the later rows read
		const void *src[kLpwDma];
#pragma unroll
		for (int i = 0; i < kLpwDma; ++i) {
			const uint64_t x = wb + 64 * i + l;
			const uint64_t before = __ballot(ne && cs < wb + 64 * i); // packets started before this row
			const int carry = before ? 64 - __builtin_clzll(before) : 0; // last such lane + 1
			const uint32_t m = wave_max_scan_dpp(own[64 * i + l]);
			const int o = (int)(m > (uint32_t)carry ? m : (uint32_t)carry) - 1;
			const uint64_t d = dls[o > 0 ? o : 0];
			src[i] = x < E ? reinterpret_cast<const void *>((d + x) << 4) : zero;
		}
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // the table is read: the slot may be refilled
#pragma unroll
		for (int i = 0; i < kLpwDma; ++i)
			glds16_nt(src[i], base + 1024 * i);
	} else {
#pragma unroll
		for (int i = 0; i < kLpwDma; ++i) {
#if CGCK_LPW_SLOTMAJOR
			const uint64_t c = wb + 8 * l + i; // lane l's 8 chunks land at +16 l of each KiB
#else
			const uint64_t c = wb + 64 * i + l;
#endif
			glds16_nt(live && c < E ? reinterpret_cast<const void *>(c << 4) : zero, base + 1024 * i);
		}
	}
	const uint64_t doff = 12 * dfirst + 16 * (uint64_t)l;
	const bool dok = DESC && dlive && l < 48 && doff < 12 * p.n;
	glds16_nt(dok ? reinterpret_cast<const void *>(reinterpret_cast<const uint8_t *>(p.desc) + doff) : zero,
		  __builtin_amdgcn_readfirstlane(lds_dslot));
}

template <bool DESC>
__device__ __forceinline__ DescW lpw_desc_lds(const uint8_t *dslot)
{
	DescW d{0, 0, 0};
	if (DESC) {
		const uint32_t *q = reinterpret_cast<const uint32_t *>(dslot) + 3 * (threadIdx.x & 63);
		d.lo = q[0];
		d.hi = q[1];
		d.w2 = q[2];
	}
	return d;
}

template <bool DESC, int C, bool W>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(W ? 4 : 1))) void lpw_kernel(KParams p)
{
	extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
	uint8_t *dring = smem + 2 * kLpwSlot; // 2 x 1 KiB descriptor slots (64 lanes x 16 B; 768 B used)
	uint32_t *so = reinterpret_cast<uint32_t *>(dring + 2 * 1024);
	uint8_t *sv = reinterpret_cast<uint8_t *>(so + C * 64);
	const int l = threadIdx.x & 63;
	const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem);
	const uint32_t ldsd = lds0 + 2 * kLpwSlot;
	const uint8_t *zero = (const uint8_t *)p.zero + (blockIdx.x & 63) * 64;
	const uint64_t NS = (p.n + 63) / 64, NC = (NS + C - 1) / C, G = gridDim.x, b = blockIdx.x;
	if (b >= NC)
		return;
	const uint64_t nsteps = (NC - b + G - 1) / G * C;
	auto gstep = [&](uint64_t j) { return (b + (j / C) * G) * C + j % C; };
	auto first_of = [&](uint64_t j) { return j < nsteps ? gstep(j) * 64 : p.n; };

	if (W && __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 1) {
		// The writer wave (as dstr_kernel's): wave 0 stages a chunk's outputs
		// and verdicts and hands them over at barrier H; this wave reads them
		// into registers, releases the staging at barrier R (wave 0 meets it
		// just before its first staging write of the next chunk) and stores
		// them, so no output store sits in wave 0's in-order vmcnt (IMIX: the
		// flush alone cost 3-7 points, profiles/r02/imix/README.md).
		const uint64_t KD = nsteps / C;
		for (uint64_t k = 0; k < KD; ++k) {
			wg_barrier(); // H_k
			const uint64_t f0 = gstep(k * C) * 64;
			const uint64_t cntp = f0 < p.n ? (p.n - f0 < (uint64_t)C * 64 ? p.n - f0 : (uint64_t)C * 64) : 0;
			uint32_t vo[C];
			uint8_t vv[C];
#pragma unroll
			for (int i = 0; i < C; ++i) {
				vo[i] = so[64 * i + l];
				vv[i] = p.verdict ? sv[64 * i + l] : 0;
			}
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
			if (k + 1 < KD)
				wg_barrier(); // R_k: the staging is free
#pragma unroll
			for (int i = 0; i < C; ++i) {
				if ((uint64_t)(64 * i + l) < cntp) {
					if (p.out)
						gbl(p.out)[f0 + 64 * i + l] = vo[i];
					if (p.verdict)
						gbl(p.verdict)[f0 + 64 * i + l] = vv[i];
				}
			}
		}
		return;
	}

	LpwStep cur = lpw_step<DESC>(p, first_of(0), load_desc<DESC>(p, first_of(0) + l, p.n));
	LpwStep nxt = lpw_step<DESC>(p, first_of(1), load_desc<DESC>(p, first_of(1) + l, p.n));
	LpwStep nn = nxt;
	uint32_t kiss = 0;      // rounds issued (round k uses data slot k & 1)
	// A full chunk's outputs leave as one 16-byte store per lane (C = 4: 256
	// outputs) issued right AFTER the next DMA round, whose wait then leaves
	// it in flight (vmcnt + 1): the store has a whole round to complete before
	// a wait must cover it.  Stored at the end of its chunk instead (in front
	// of the next round in the in-order vmcnt), the flush cost IMIX 3-7 points
	// (profiles/r02/imix/README.md).  Lab mode 6: the end-of-chunk flush.
	static_assert(C % 4 == 0, "C / 4 16-byte stores per lane per chunk");
	const bool defer_ok = !W && p.out && !p.verdict && (reinterpret_cast<uintptr_t>(p.out) & 15) == 0 &&
			      p.contig != 6 && p.contig != 5;
	bool pend = false; // a chunk's outputs wait in the staging for the next round
	int sage = 0;      // waits left that may leave the chunk store in flight
	uint64_t pf0 = 0;  // its first packet
	bool pre = false;       // cur's window 0 (with step j + 2's descriptors) already issued
	for (uint64_t j = 0; j < nsteps; ++j) {
		const uint64_t first = first_of(j);
		uint32_t acc = 0, corr = 0;
		Hdr h{};
		if (first < p.n && cur.nwin > 0) {
			// the header's chunks, loop-carried in native vectors (an array of
			// uint4, a union type, was put in scratch)
			u32x4_t t8[8];
#pragma unroll
			for (int u = 0; u < 8; ++u)
				t8[u] = u32x4_t{0, 0, 0, 0};
			if (!pre) {
				lpw_issue<DESC>(p, cur.S, cur.E, true, cur.gather, cur.cs, cur.ce, cur.dl, smem + (kiss & 1) * kLpwSlot,
						lds0 + (kiss & 1) * kLpwSlot, first_of(j + 2), first_of(j + 2) < p.n,
						ldsd + (uint32_t)((j + 2) & 1) * 1024, zero);
				++kiss;
			}
			for (uint32_t t = 0; t < cur.nwin; ++t) {
				// the next round: this step's next window, or the next step's first
				// (carrying the descriptors of step j + 3)
				const bool more = t + 1 < cur.nwin;
				const bool nx = !more && first_of(j + 1) < p.n && nxt.nwin > 0;
				const uint64_t iwb = more ? cur.S + (uint64_t)(t + 1) * kLpwWin : nxt.S;
				const uint64_t iE = more ? cur.E : nxt.E;
				lpw_issue<DESC>(p, iwb, iE, more || nx, more ? cur.gather : nxt.gather, more ? cur.cs : nxt.cs,
						more ? cur.ce : nxt.ce, more ? cur.dl : nxt.dl, smem + (kiss & 1) * kLpwSlot,
						lds0 + (kiss & 1) * kLpwSlot, first_of(j + 3), !more && first_of(j + 3) < p.n,
						ldsd + (uint32_t)((j + 3) & 1) * 1024, zero);
				++kiss;
				pre = nx;
				if (pend) {
					const __amdgpu_buffer_rsrc_t rs = out_rsrc(p.out + pf0, C * 256);
#pragma unroll
					for (int i = 0; i < C / 4; ++i)
						bstore16<kSc1>(rs, 16 * (64 * i + l), reinterpret_cast<const u32x4_t *>(so)[64 * i + l]);
					pend = false;
					sage = 2;
				}
				// The wait for the previous round.  A store issued after this
				// round (sage 2) or after the previous one (sage 1) may stay in
				// flight: it sits between the two rounds in the in-order count.
				if (sage > 0) {
					--sage;
					asm volatile("s_waitcnt vmcnt(%0)" ::"i"(kLpwDma + 1 + C / 4) : "memory");
				} else {
					asm volatile("s_waitcnt vmcnt(%0)" ::"i"(kLpwDma + 1) : "memory");
				}
				// (the covering vmcnt alone orders this wave's reads behind its
				// DMA; the barrier is kept in the one-wave form as measured)
				if (!W)
					__builtin_amdgcn_s_barrier();
				if (t == 0) // step j + 2's descriptors came with window 0 of this step
					nn = lpw_step<DESC>(p, first_of(j + 2), lpw_desc_lds<DESC>(dring + ((j + 2) & 1) * 1024));
				if (p.contig == 4) // lab $CGCK_LPW_NOCONS: rounds without the per-window work
					continue;
				const uint4 *win = reinterpret_cast<const uint4 *>(smem + (kiss & 1) * kLpwSlot); // round kiss - 2
				const uint64_t wb = cur.S + (uint64_t)t * kLpwWin;
				const uint64_t we = wb + kLpwWin;
				// 1. reads of single chunks: the packet's edge chunks and its
				// header chunks cs .. cs + 7 that fall in this window (kept in
				// registers across windows; the header is read once per step)
				const bool head = cur.ok && cur.nch > 0 && cur.cs >= wb && cur.cs < we;
				const bool tail = cur.ok && cur.nch > 0 && cur.ce - 1 >= wb && cur.ce - 1 < we;
				const bool dw = !__any(cur.ok && ((cur.q | cur.len) & 3) != 0);
				if (__any(head && cur.q != 0))
					corr += head && cur.q != 0 ? lead_sum(win[lpw_at((int)(cur.cs - wb))], cur.q, dw) : 0u;
				if (__any(tail && cur.e != 16))
					corr += tail && cur.e != 16 ? trail_sum(win[lpw_at((int)(cur.ce - 1 - wb))], cur.e, dw) : 0u;
				const bool hwin = cur.ok && cur.cs + 8 > wb && cur.cs < we;
				if (!(p.flags & CGCK_RAW) && __any(hwin)) {
					const u32x4_t *win4 = reinterpret_cast<const u32x4_t *>(win);
#pragma unroll
					for (int u = 0; u < 8; ++u) {
						const uint64_t c = cur.cs + u;
						const bool in = hwin && c >= wb && c < we;
						const u32x4_t c8 = win4[in ? lpw_at((int)(c - wb)) : 0];
						t8[u] = in ? c8 : t8[u];
					}
				}
				// 2. lane per chunk: every owned chunk's sum (conflict-free 16-byte
				// reads), prefix-summed over the window in lane order; the rows'
				// scans are independent, their carries added after.  The prefix is
				// written over the slot's first rows, already read.
#if CGCK_LPW_SLOTMAJOR
				static_assert(kLpwDma == 8, "slot-major windows are 64 lanes x 8 chunks");
				// lane l owns chunks [8 l, 8 l + 8): local prefix, one wave scan
				uint32_t xs[8];
				uint32_t run = 0;
#pragma unroll
				for (int i = 0; i < 8; ++i) {
					const uint4 v = win[64 * i + l];
					run += wb + 8 * l + i < cur.E ? sum4(v, 0u) : 0u;
					xs[i] = run;
				}
				const uint32_t before = wave_scan_dpp(run) - run;
				asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // every read of the slot's chunks is done
				uint32_t *pfx = reinterpret_cast<uint32_t *>(smem + (kiss & 1) * kLpwSlot);
				{
					typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
					u32x4v *p4 = reinterpret_cast<u32x4v *>(pfx + 8 * l);
					p4[0] = u32x4v{before + xs[0], before + xs[1], before + xs[2], before + xs[3]};
					p4[1] = u32x4v{before + xs[4], before + xs[5], before + xs[6], before + xs[7]};
				}
#elif CGCK_LPW_PAIR
				// A lane per PAIR of chunks (2 l, 2 l + 1 of each 2 KiB row
				// pair): half the wave scans of a lane per chunk (4 a window
				// instead of 8: the scans' DPP chain was the window's largest
				// issue cost, lpw being issue-bound on the packed layout —
				// SQ_ACTIVE_INST_ANY 0.49 of its wave cycles against dstr's
				// 0.20, profiles/r06/lpwpmc/).  The two 16-byte reads of a
				// lane go first / second by bit 3 of the lane, so lanes l and
				// l + 8 (32 bytes apart x 8) never hit the same banks.
				uint32_t ya[kLpwDma / 2], yb[kLpwDma / 2];
				const int sw = (l >> 3) & 1;
#pragma unroll
				for (int r = 0; r < kLpwDma / 2; ++r) {
					const int c = 128 * r + 2 * l;
					const uint4 va = win[c + sw], vb = win[c + 1 - sw];
					const uint32_t sa = wb + (uint64_t)(c + sw) < cur.E ? sum4(va, 0u) : 0u;
					const uint32_t sb = wb + (uint64_t)(c + 1 - sw) < cur.E ? sum4(vb, 0u) : 0u;
					const uint32_t s1 = sw ? sa : sb; // chunk c + 1's sum
					const uint32_t inc = wave_scan_dpp(sa + sb);
					yb[r] = inc;
					ya[r] = inc - s1;
				}
				asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // every read of the slot's chunks is done
				uint32_t *pfx = reinterpret_cast<uint32_t *>(smem + (kiss & 1) * kLpwSlot);
				uint32_t carry = 0;
#pragma unroll
				for (int r = 0; r < kLpwDma / 2; ++r) {
					typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
					*reinterpret_cast<u32x2v *>(pfx + 128 * r + 2 * l) = u32x2v{ya[r] + carry, yb[r] + carry};
					carry += __builtin_amdgcn_readlane(yb[r], 63);
				}
#else
				uint32_t xs[kLpwDma];
#pragma unroll
				for (int r = 0; r < kLpwDma; ++r) {
					const uint4 v = win[64 * r + l];
					xs[r] = wave_scan_dpp(wb + 64 * r + l < cur.E ? sum4(v, 0u) : 0u);
				}
				asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // every read of the slot's chunks is done
				uint32_t *pfx = reinterpret_cast<uint32_t *>(smem + (kiss & 1) * kLpwSlot);
				uint32_t carry = 0;
#pragma unroll
				for (int r = 0; r < kLpwDma; ++r) {
					pfx[64 * r + l] = xs[r] + carry;
					carry += __builtin_amdgcn_readlane(xs[r], 63);
				}
#endif
				// 3. lane per packet: its chunks in this window as a prefix difference
				const uint64_t lo = cur.cs > wb ? cur.cs : wb;
				const uint64_t hi = cur.ce < we ? cur.ce : we;
				if (cur.ok && hi > lo)
					acc += pfx[(int)(hi - 1 - wb)] - (lo > wb ? pfx[(int)(lo - 1 - wb)] : 0u);
				asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // the slots are refilled next round
			}
			if (!(p.flags & CGCK_RAW)) {
				uint4 w8[8];
#pragma unroll
				for (int u = 0; u < 8; ++u)
					w8[u] = make_uint4(t8[u].x, t8[u].y, t8[u].z, t8[u].w);
				h = header<8, false>(w8, reinterpret_cast<const uint4 *>(cur.a0 & ~(uint64_t)15), cur.nch, cur.q,
						     cur.len, p.flags, cur.ok);
			}
			if (!pre) { // the last round was a zero round: drained before the next issue or a fallback
				asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
				sage = 0; // (a looser count would no longer cover a round)
			}
		} else if (first < p.n) {
			// not chained: the lane's packet straight from global memory
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			sage = 0;
			pre = false;
			nn = lpw_step<DESC>(p, first_of(j + 2), load_desc<DESC>(p, first_of(j + 2) + l, p.n));
			const uint4 *c0 = reinterpret_cast<const uint4 *>(cur.a0 & ~(uint64_t)15);
			const int cnt = cur.ok ? cur.nch : 0;
			for (int i = 0; __any(i < cnt); ++i) {
				const uint4 v = ldc<false>(c0, i, cnt, p.zero);
				acc = i < cnt ? sum4(v, acc) : acc;
				if (i == 0 && cnt > 0 && cur.q != 0)
					corr += lead_sum(v, cur.q, false);
				if (i == cnt - 1 && cur.e != 16)
					corr += trail_sum(v, cur.e, false);
			}
			if (!(p.flags & CGCK_RAW)) {
				uint4 w8[8];
#pragma unroll
				for (int u = 0; u < 8; ++u)
					w8[u] = ldc<false>(c0, u, cnt, p.zero);
				h = header<8, false>(w8, c0, cur.nch, cur.q, cur.len, p.flags, cur.ok);
			}
		}
		if (W && j % C == 0 && j > 0)
			wg_barrier(); // R: the writer has read the last chunk's staging
		if (pend) { // no round came (a fallback or an empty step): flush before the staging is reused
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
			for (int i = l; i < C * 64; i += 64)
				gbl(p.out)[pf0 + i] = so[i];
			pend = false;
		}
		if (first < p.n) {
			const uint32_t r = fold16(acc) + (0xffffu - fold16(corr));
			const Res res = result(p, cur.a0, cur.len, fold16(r), h);
			const int slot = (int)(j % C) * 64 + l;
			so[slot] = res.out;
			if (p.verdict) // (the verdict staging is allocated only with verdicts)
				sv[slot] = (uint8_t)res.verdict;
		}
		if (W && (j + 1) % C == 0) {
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // the chunk's outputs are in LDS
			wg_barrier();                                      // H: hand them to the writer
		} else if (!W && ((j + 1) % C == 0 || j + 1 == nsteps) && p.contig != 5) { // lab mode 5: no flush
			// flush the chunk's outputs (packets [f0, f0 + 64 C) of the batch)
			const uint64_t f0 = gstep(j - j % C) * 64;
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
			const uint64_t cntp = f0 < p.n ? (p.n - f0 < (uint64_t)C * 64 ? p.n - f0 : (uint64_t)C * 64) : 0;
			if (defer_ok && cntp == (uint64_t)C * 64 && j + 1 < nsteps) {
				pend = true; // stored after the next round's issue
				pf0 = f0;
			} else {
				for (uint64_t i = l; i < cntp; i += 64) {
					if (p.out)
						gbl(p.out)[f0 + i] = so[i];
					if (p.verdict)
						gbl(p.verdict)[f0 + i] = sv[i];
				}
			}
		}
		cur = nxt;
		nxt = nn;
	}
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

#if CGCK_LAB
// lpx: lpw with TWO rounds in flight.  lpw waits for round r - 1 right after
// issuing round r, so one 8 KiB window per wave is in flight while a window is
// reduced (its DMA rounds alone: 76.8 % of 8 TB/s).  Here a round's slot is
// refilled as soon as the window's bytes are in registers (dstr's trick): the
// wave waits for round r, reads the window (chunk sums, edge chunks, header
// chunks), issues round r + 2 into the same slot, and only then scans; the
// prefix goes to a separate 2 KiB area.  Every step has at least one round (a
// zero round for a step computed from global memory or past the batch), so
// the issue cursor runs exactly two rounds ahead through cur / nxt / nn; round
// (k, 0) carries the descriptors of step k + 2, which processing (k, 0) turns
// into nn before the round after it can need them.  22.3 KiB of LDS: 7 waves
// per CU, 112 KiB in flight per CU against lpw's 64.
template <bool DESC, int C>
__global__ __launch_bounds__(64) void lpx_kernel(KParams p)
{
	extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
	// 2 x 1 KiB descriptor slots and a third the rounds without descriptors
	// write their zero line into (round (k, 0)'s descriptors of step k + 2 wait
	// in their slot while later rounds of step k are issued)
	uint8_t *dring = smem + 2 * kLpwSlot;
	uint32_t *pfx = reinterpret_cast<uint32_t *>(dring + 3 * 1024); // kLpwWin prefix sums
	uint32_t *so = pfx + kLpwWin;
	uint8_t *sv = reinterpret_cast<uint8_t *>(so + C * 64);
	const int l = threadIdx.x & 63;
	const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem);
	const uint32_t ldsd = lds0 + 2 * kLpwSlot;
	const uint8_t *zero = (const uint8_t *)p.zero + (blockIdx.x & 63) * 64;
	const uint64_t NS = (p.n + 63) / 64, NC = (NS + C - 1) / C, G = gridDim.x, b = blockIdx.x;
	if (b >= NC)
		return;
	const uint64_t nsteps = (NC - b + G - 1) / G * C;
	auto gstep = [&](uint64_t j) { return (b + (j / C) * G) * C + j % C; };
	auto first_of = [&](uint64_t j) { return j < nsteps ? gstep(j) * 64 : p.n; };

	LpwStep cur = lpw_step<DESC>(p, first_of(0), load_desc<DESC>(p, first_of(0) + l, p.n));
	LpwStep nxt = lpw_step<DESC>(p, first_of(1), load_desc<DESC>(p, first_of(1) + l, p.n));
	LpwStep nn = nxt; // step j + 2: from the descriptors round (j, 0) carries, at processing (j, 0)
	uint32_t kiss = 0; // rounds issued (round k uses data slot k & 1)
	int ia = 0;        // issue cursor: step j + ia ...
	uint32_t iw = 0;   // ... window iw
	auto rounds = [](uint32_t nwin) { return nwin ? nwin : 1u; };
	// issue the round at the cursor (one call site per step struct: a selected
	// struct or field would put the structs in scratch), then advance it
#define CGCK_LPX_ISSUE(ST, K)                                                                            \
	do {                                                                                             \
		const uint64_t k_ = (K);                                                                \
		lpw_issue<DESC>(p, ST.S + (uint64_t)iw * kLpwWin, ST.E, ST.nwin > 0 && first_of(k_) < p.n, ST.gather, \
				ST.cs, ST.ce, ST.dl, smem + (kiss & 1) * kLpwSlot, lds0 + (kiss & 1) * kLpwSlot,      \
				first_of(k_ + 2), iw == 0 && first_of(k_ + 2) < p.n,                           \
				ldsd + (iw == 0 ? (uint32_t)((k_ + 2) & 1) : 2u) * 1024, zero);               \
		++kiss;                                                                                 \
		if (iw + 1 < rounds(ST.nwin)) {                                                          \
			++iw;                                                                           \
		} else {                                                                                \
			++ia;                                                                           \
			iw = 0;                                                                         \
		}                                                                                       \
	} while (0)
	auto issue_next = [&](uint64_t j) __attribute__((always_inline)) {
		if (ia == 0)
			CGCK_LPX_ISSUE(cur, j);
		else if (ia == 1)
			CGCK_LPX_ISSUE(nxt, j + 1);
		else
			CGCK_LPX_ISSUE(nn, j + 2);
	};
	issue_next(0);
	issue_next(0);
	static_assert(C % 4 == 0, "C / 4 16-byte stores per lane per chunk");
	const bool defer_ok = p.out && !p.verdict && (reinterpret_cast<uintptr_t>(p.out) & 15) == 0;
	bool pend = false; // a chunk's outputs wait in the staging for the next round
	int sage = 0;      // waits left that may leave the chunk store in flight
	uint64_t pf0 = 0;
	for (uint64_t j = 0; j < nsteps; ++j) {
		const uint64_t first = first_of(j);
		const bool live = first < p.n && cur.nwin > 0;
		uint32_t acc = 0, corr = 0;
		Hdr h{};
		u32x4_t t8[8];
#pragma unroll
		for (int u = 0; u < 8; ++u)
			t8[u] = u32x4_t{0, 0, 0, 0};
		const uint32_t R = rounds(cur.nwin);
		for (uint32_t t = 0; t < R; ++t) {
			// round (j, t); issued after it: the next round, and a chunk store
			// (after this round: two waits leave it in flight)
			if (sage > 0) {
				--sage;
				asm volatile("s_waitcnt vmcnt(%0)" ::"i"(kLpwDma + 1 + C / 4) : "memory");
			} else {
				asm volatile("s_waitcnt vmcnt(%0)" ::"i"(kLpwDma + 1) : "memory");
			}
			if (t == 0)
				nn = lpw_step<DESC>(p, first_of(j + 2), lpw_desc_lds<DESC>(dring + ((j + 2) & 1) * 1024));
			const uint4 *win = reinterpret_cast<const uint4 *>(smem + (kiss & 1) * kLpwSlot); // round kiss - 2
			const uint64_t wb = cur.S + (uint64_t)t * kLpwWin;
			const uint64_t we = wb + kLpwWin;
			uint32_t cs8[kLpwDma];
			if (live) {
				const bool head = cur.ok && cur.nch > 0 && cur.cs >= wb && cur.cs < we;
				const bool tail = cur.ok && cur.nch > 0 && cur.ce - 1 >= wb && cur.ce - 1 < we;
				const bool dw = !__any(cur.ok && ((cur.q | cur.len) & 3) != 0);
				if (__any(head && cur.q != 0))
					corr += head && cur.q != 0 ? lead_sum(win[(int)(cur.cs - wb)], cur.q, dw) : 0u;
				if (__any(tail && cur.e != 16))
					corr += tail && cur.e != 16 ? trail_sum(win[(int)(cur.ce - 1 - wb)], cur.e, dw) : 0u;
				const bool hwin = cur.ok && cur.cs + 8 > wb && cur.cs < we;
				if (!(p.flags & CGCK_RAW) && __any(hwin)) {
					const u32x4_t *win4 = reinterpret_cast<const u32x4_t *>(win);
#pragma unroll
					for (int u = 0; u < 8; ++u) {
						const uint64_t c = cur.cs + u;
						const bool in = hwin && c >= wb && c < we;
						const u32x4_t c8 = win4[in ? (int)(c - wb) : 0];
						t8[u] = in ? c8 : t8[u];
					}
				}
#pragma unroll
				for (int r = 0; r < kLpwDma; ++r) {
					const uint4 v = win[64 * r + l];
					cs8[r] = wb + 64 * r + l < cur.E ? sum4(v, 0u) : 0u;
				}
			}
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // the window is in registers: refill its slot
			issue_next(j);
			if (pend) {
				const __amdgpu_buffer_rsrc_t rs = out_rsrc(p.out + pf0, C * 256);
#pragma unroll
				for (int i = 0; i < C / 4; ++i)
					bstore16<kSc1>(rs, 16 * (64 * i + l), reinterpret_cast<const u32x4_t *>(so)[64 * i + l]);
				pend = false;
				sage = 2;
			}
			if (live) {
				uint32_t carry = 0;
#pragma unroll
				for (int r = 0; r < kLpwDma; ++r) {
					const uint32_t xs = wave_scan_dpp(cs8[r]);
					pfx[64 * r + l] = xs + carry;
					carry += __builtin_amdgcn_readlane(xs, 63);
				}
				const uint64_t lo = cur.cs > wb ? cur.cs : wb;
				const uint64_t hi = cur.ce < we ? cur.ce : we;
				if (cur.ok && hi > lo)
					acc += pfx[(int)(hi - 1 - wb)] - (lo > wb ? pfx[(int)(lo - 1 - wb)] : 0u);
				asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // the prefix area is rewritten next round
			}
		}
		if (live) {
			if (!(p.flags & CGCK_RAW)) {
				uint4 w8[8];
#pragma unroll
				for (int u = 0; u < 8; ++u)
					w8[u] = make_uint4(t8[u].x, t8[u].y, t8[u].z, t8[u].w);
				h = header<8, false>(w8, reinterpret_cast<const uint4 *>(cur.a0 & ~(uint64_t)15), cur.nch, cur.q,
						     cur.len, p.flags, cur.ok);
			}
		} else if (first < p.n) {
			// no window covers the step (more than 16 windows): the lane's packet
			// straight from global memory, after a drain (the two rounds in
			// flight complete first; the counts after it only over-wait)
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			sage = 0;
			const uint4 *c0 = reinterpret_cast<const uint4 *>(cur.a0 & ~(uint64_t)15);
			const int cnt = cur.ok ? cur.nch : 0;
			for (int i = 0; __any(i < cnt); ++i) {
				const uint4 v = ldc<false>(c0, i, cnt, p.zero);
				acc = i < cnt ? sum4(v, acc) : acc;
				if (i == 0 && cnt > 0 && cur.q != 0)
					corr += lead_sum(v, cur.q, false);
				if (i == cnt - 1 && cur.e != 16)
					corr += trail_sum(v, cur.e, false);
			}
			if (!(p.flags & CGCK_RAW)) {
				uint4 w8[8];
#pragma unroll
				for (int u = 0; u < 8; ++u)
					w8[u] = ldc<false>(c0, u, cnt, p.zero);
				h = header<8, false>(w8, c0, cur.nch, cur.q, cur.len, p.flags, cur.ok);
			}
		}
		if (first < p.n) {
			const uint32_t r = fold16(acc) + (0xffffu - fold16(corr));
			const Res res = result(p, cur.a0, cur.len, fold16(r), h);
			const int slot = (int)(j % C) * 64 + l;
			so[slot] = res.out;
			if (p.verdict)
				sv[slot] = (uint8_t)res.verdict;
		}
		if ((j + 1) % C == 0 || j + 1 == nsteps) {
			const uint64_t f0 = gstep(j - j % C) * 64;
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
			const uint64_t cntp = f0 < p.n ? (p.n - f0 < (uint64_t)C * 64 ? p.n - f0 : (uint64_t)C * 64) : 0;
			if (defer_ok && cntp == (uint64_t)C * 64 && j + 1 < nsteps) {
				pend = true; // stored after the next round's issue
				pf0 = f0;
			} else {
				for (uint64_t i = l; i < cntp; i += 64) {
					if (p.out)
						gbl(p.out)[f0 + i] = so[i];
					if (p.verdict)
						gbl(p.verdict)[f0 + i] = sv[i];
				}
			}
		}
		cur = nxt;
		nxt = nn;
		--ia;
	}
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#undef CGCK_LPX_ISSUE
}
#endif

bool lpw_ok(const KParams &p)
{
	return !p.bad && !(p.flags & (CGCK_STORE | kFlagNoLenCheck | kFlagL4Auto)) &&
	       (reinterpret_cast<uintptr_t>(p.desc) & 15) == 0;
}

hipError_t launch_lpw(const KParams &p, int num_cus, hipStream_t st)
{
	static const int wpc = [] { // $CGCK_LPW_WPC: waves per CU
		const char *e = CGCK_ENV("CGCK_LPW_WPC");
		return e && atoi(e) > 0 ? atoi(e) : 8;
	}();
	KParams q = p;
	q.contig = 0;
#if CGCK_LAB
	static const bool nocons = CGCK_ENV("CGCK_LPW_NOCONS") != nullptr;
	static const bool noflush = CGCK_ENV("CGCK_LPW_NOFLUSH") != nullptr;
	static const bool nodefer = CGCK_ENV("CGCK_LPW_NODEFER") != nullptr; // the end-of-chunk flush
	if (nocons)
		q.contig = 4;
	else if (noflush)
		q.contig = 5;
	else if (nodefer)
		q.contig = 6;
#endif
	constexpr int C = 4; // 8 KiB windows: 19.3 KiB of LDS per workgroup, 8 per CU
	const uint64_t want = (p.n + 64 * C - 1) / (64 * C);
	const uint64_t cap = (uint64_t)num_cus * wpc;
	const dim3 g((unsigned)(want < cap ? (want ? want : 1) : cap));
	const size_t lds = 2 * kLpwSlot + 2 * 1024 + C * 64 * (p.verdict ? 5 : 4);
#define CGCK_LPW(DD, WW)                                                                  \
	do {                                                                              \
		CGCK_NOTE_KERNEL("lpw_kernel<%s, %d, %s>", tf(DD), C, tf(WW));              \
		hipLaunchKernelGGL((lpw_kernel<DD, C, WW>), g, dim3((WW) ? 128 : 64), lds, st, q); \
	} while (0)
#if CGCK_LAB
	// $CGCK_LPW_C=8: chunks of 8 steps for batches without verdicts (20 KiB
	// of LDS per workgroup)
	static const bool c8 = CGCK_ENV("CGCK_LPW_C") && atoi(CGCK_ENV("CGCK_LPW_C")) == 8;
	if (c8 && !p.verdict) {
		constexpr int C8 = 8;
		const uint64_t want8 = (p.n + 64 * C8 - 1) / (64 * C8);
		const dim3 g8((unsigned)(want8 < cap ? (want8 ? want8 : 1) : cap));
		const size_t lds8 = 2 * kLpwSlot + 2 * 1024 + C8 * 64 * 4;
		if (p.desc) {
			CGCK_NOTE_KERNEL("lpw_kernel<true, 8, false>");
			hipLaunchKernelGGL((lpw_kernel<true, C8, false>), g8, dim3(64), lds8, st, q);
		} else {
			CGCK_NOTE_KERNEL("lpw_kernel<false, 8, false>");
			hipLaunchKernelGGL((lpw_kernel<false, C8, false>), g8, dim3(64), lds8, st, q);
		}
		return hipGetLastError();
	}
	// $CGCK_LPW_X=1: lpx_kernel, two rounds in flight (7 waves per CU)
	static const bool two = CGCK_ENV("CGCK_LPW_X") && atoi(CGCK_ENV("CGCK_LPW_X")) != 0;
	if (two) {
		static const int wpcx = [] {
			const char *e = CGCK_ENV("CGCK_LPX_WPC");
			return e && atoi(e) > 0 ? atoi(e) : 7;
		}();
		const uint64_t capx = (uint64_t)num_cus * wpcx;
		const dim3 gx((unsigned)(want < capx ? (want ? want : 1) : capx));
		const size_t ldsx = 2 * kLpwSlot + 3 * 1024 + 4 * kLpwWin + C * 64 * (p.verdict ? 5 : 4);
		if (p.desc) {
			CGCK_NOTE_KERNEL("lpx_kernel<true, %d>", C);
			hipLaunchKernelGGL((lpx_kernel<true, C>), gx, dim3(64), ldsx, st, q);
		} else {
			CGCK_NOTE_KERNEL("lpx_kernel<false, %d>", C);
			hipLaunchKernelGGL((lpx_kernel<false, C>), gx, dim3(64), ldsx, st, q);
		}
		return hipGetLastError();
	}
	// $CGCK_LPW_W=1: the writer wave (lost: capped at 128 VGPRs it spills,
	// 52.5-53.7 % vs 70.3-70.4 %, profiles/r02/imix/README.md)
	static const bool wr = CGCK_ENV("CGCK_LPW_W") && atoi(CGCK_ENV("CGCK_LPW_W")) != 0;
	if (wr) {
		if (p.desc)
			CGCK_LPW(true, true);
		else
			CGCK_LPW(false, true);
		return hipGetLastError();
	}
#endif
	if (p.desc)
		CGCK_LPW(true, false);
	else
		CGCK_LPW(false, false);
#undef CGCK_LPW
	return hipGetLastError();
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
	if (nt) {
		CGCK_NOTE_KERNEL("lpp_kernel<%s, true, %d, %s>", tf(DESC), S0, tf(CLAMP));
		hipLaunchKernelGGL((lpp_kernel<DESC, true, S0, CLAMP>), dim3(blocks), dim3(256), 0, st, p);
	} else {
		CGCK_NOTE_KERNEL("lpp_kernel<%s, false, %d, %s>", tf(DESC), S0, tf(CLAMP));
		hipLaunchKernelGGL((lpp_kernel<DESC, false, S0, CLAMP>), dim3(blocks), dim3(256), 0, st, p);
	}
	return hipGetLastError();
}

// shape: 0 = 4 chunks up front, clamped; 1 = 6 clamped; 2 = 6 predicated
// (the default, kDefaultLppShape; the only one in libcgck.so); 3 = 4 predicated
hipError_t launch_lpp(const KParams &p, int num_cus, bool nt, int shape, hipStream_t st)
{
	const int mb = num_cus * 8;
	const bool d = p.desc != nullptr;
	switch (shape) {
#if CGCK_LAB
	case 1:
		return d ? launch_lpp_t<true, 6, true>(p, mb, nt, st) : launch_lpp_t<false, 6, true>(p, mb, nt, st);
	case 3:
		return d ? launch_lpp_t<true, 4, false>(p, mb, nt, st) : launch_lpp_t<false, 4, false>(p, mb, nt, st);
	case 0:
		return d ? launch_lpp_t<true, 4, true>(p, mb, nt, st) : launch_lpp_t<false, 4, true>(p, mb, nt, st);
#endif
	default:
		return d ? launch_lpp_t<true, 6, false>(p, mb, nt, st) : launch_lpp_t<false, 6, false>(p, mb, nt, st);
	}
}

template <bool DESC>
static hipError_t launch_slot2_t(const KParams &p, int max_blocks, bool nt, hipStream_t st)
{
	uint64_t want = (p.n + 4 * 64 - 1) / (4 * 64);
	int blocks = (int)(want < (uint64_t)max_blocks ? want : (uint64_t)max_blocks);
	if (blocks < 1)
		blocks = 1;
	if (nt) {
		CGCK_NOTE_KERNEL("slot2_kernel<%s, true>", tf(DESC));
		hipLaunchKernelGGL((slot2_kernel<DESC, true>), dim3(blocks), dim3(256), 0, st, p);
	} else {
		CGCK_NOTE_KERNEL("slot2_kernel<%s, false>", tf(DESC));
		hipLaunchKernelGGL((slot2_kernel<DESC, false>), dim3(blocks), dim3(256), 0, st, p);
	}
	return hipGetLastError();
}

hipError_t launch_slot2(const KParams &p, int num_cus, bool nt, hipStream_t st)
{
	// 8 blocks per CU requested; 41 KiB of LDS per block (the 2048-packet
	// output windows) keeps 3 resident per CU — 1984-packet windows (4
	// resident) and 3072 (2) measured the same.  $CGCK_BPC overrides the
	// blocks per CU for A/B runs.
	static const int bpc = [] {
		const char *e = CGCK_ENV("CGCK_BPC");
		return e && atoi(e) > 0 ? atoi(e) : 8;
	}();
	const int mb = num_cus * bpc;
	return p.desc ? launch_slot2_t<true>(p, mb, nt, st) : launch_slot2_t<false>(p, mb, nt, st);
}

#if CGCK_LAB
template <bool DESC>
static hipError_t launch_slot_t(const KParams &p, int max_blocks, bool nt, hipStream_t st)
{
	// each wave owns a contiguous packet range of >= ~64 packets
	uint64_t want = (p.n + 4 * 64 - 1) / (4 * 64);
	int blocks = (int)(want < (uint64_t)max_blocks ? want : (uint64_t)max_blocks);
	if (blocks < 1)
		blocks = 1;
	if (nt) {
		CGCK_NOTE_KERNEL("slot_kernel<%s, true>", tf(DESC));
		hipLaunchKernelGGL((slot_kernel<DESC, true>), dim3(blocks), dim3(256), 0, st, p);
	} else {
		CGCK_NOTE_KERNEL("slot_kernel<%s, false>", tf(DESC));
		hipLaunchKernelGGL((slot_kernel<DESC, false>), dim3(blocks), dim3(256), 0, st, p);
	}
	return hipGetLastError();
}

template <bool DESC>
static hipError_t launch_lppp_t(const KParams &p, int max_blocks, bool nt, hipStream_t st)
{
	uint64_t want = (p.n + 255) / 256;
	int blocks = (int)(want < (uint64_t)max_blocks ? want : (uint64_t)max_blocks);
	if (blocks < 1)
		blocks = 1;
	if (nt) {
		CGCK_NOTE_KERNEL("lppp_kernel<%s, true>", tf(DESC));
		hipLaunchKernelGGL((lppp_kernel<DESC, true>), dim3(blocks), dim3(256), 0, st, p);
	} else {
		CGCK_NOTE_KERNEL("lppp_kernel<%s, false>", tf(DESC));
		hipLaunchKernelGGL((lppp_kernel<DESC, false>), dim3(blocks), dim3(256), 0, st, p);
	}
	return hipGetLastError();
}

hipError_t launch_lppp(const KParams &p, int num_cus, bool nt, hipStream_t st)
{
	return p.desc ? launch_lppp_t<true>(p, num_cus * 8, nt, st) : launch_lppp_t<false>(p, num_cus * 8, nt, st);
}

hipError_t launch_slot(const KParams &p, int num_cus, bool nt, hipStream_t st)
{
	return p.desc ? launch_slot_t<true>(p, num_cus * 8, nt, st) : launch_slot_t<false>(p, num_cus * 8, nt, st);
}
#endif // CGCK_LAB

} // namespace cgck
