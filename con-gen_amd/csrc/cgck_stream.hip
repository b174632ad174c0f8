// cgck_stream.hip — dense strided batches streamed through LDS by DMA (the
// 1500 B config).
//
// Why.  On MI355X a contiguous streaming read issued as
// global_load_lds_dwordx4 with the nontemporal policy reaches 6.8-7.0 TB/s
// chip-wide against 6.2-6.5 TB/s for register loads on the same boxes
// (tools/probe.py variants 41/43/44 vs 0/1/4; MI355X_MICROARCH.md
// 'ldsdma-fill').  The per-packet lane-group loads of cgck_group.hip (four
// 256-byte segments per wave-instruction) fed through the same DMA path
// measured only 6.4 TB/s even with no arithmetic, so this kernel moves each
// step's bytes as ONE contiguous region instead.
//
// Layout.  One wave per workgroup; each wave owns a contiguous packet range
// and walks it 4 packets per step.  A step's region is the 6 KiB from the
// first packet's 16-byte-aligned start: 6 DMA instructions, lane l of
// instruction i moving bytes [1024 i + 16 l, +16) into the same place of an
// LDS slot (the region lands byte-linear in LDS).  4 consecutive packets fit
// when 3 * stride + 15 + ip_len <= 6144 (stride, ip_len <= 1520).  Lanes
// whose 16 bytes lie past the batch's last packet read a zero line instead
// (no access past the caller's buffer).
//
// Pipeline.  A ring of 3 slots per wave: issue step j+2, wait with a
// counted vmcnt for step j (12 DMA may stay in flight), s_barrier (LDS-DMA
// data is ordered for ds_read only by the issuing wave's vmcnt followed by a
// barrier), read, lgkmcnt(0) before the slot is refilled.  No global store
// inside the pipeline (it would count in vmcnt): outputs are staged in LDS
// and written per window of kStrWin steps behind a vmcnt(0).  The DMA is
// inline asm (M0 = the wave-uniform LDS base), so the compiler counts none
// of it: every wait on it is explicit here.
//
// Arithmetic (lean by construction).  Lane (g = lane / 16, gl) sums region
// chunks c0_g + 16 s + gl, s = 0..5, of packet g: interior chunks whole, the
// first chunk without its q lead bytes, the last without its tail, chunks
// past the packet dropped.  Group sums by DPP.  The header (ip_hl, ip_p and
// the ip_hl*4 header bytes, src/dst) is read straight from LDS by the
// group's lanes, and lane 0 finishes the packet as result() does.
//
// Scope: strided batches, dword-aligned packets (base, stride, l3_off),
// 20 <= ip_len <= 1520, stride <= 1520, flags RAW or any of IP / L4 /
// L4_NOPSEUDO (no field zeroing, verify or in-place store), no bad
// counters.  Everything else takes cgck_group.hip.
#include "cgck_device.h"

#include <stdlib.h>

namespace cgck {

constexpr int kStrS = 6;                    // DMA instructions (KiB) per step
#ifndef CGCK_STR_WIN
#define CGCK_STR_WIN 64
#endif
constexpr int kStrWin = CGCK_STR_WIN;       // steps per output window
constexpr uint32_t kStrSlot = kStrS * 1024; // bytes per slot

// DMA of the region of the step starting at packet `first` into a slot.
// live = false (past the window) or lanes past the batch's last chunk read
// the zero line.
__device__ __forceinline__ void str_issue(const KParams &p, uint64_t first, bool live, uint64_t last_chunk,
					  const uint8_t *zero, uint32_t lds_slot)
{
	const int lane = threadIdx.x & 63;
	const uint64_t a = (reinterpret_cast<uint64_t>(p.base) + first * p.stride + p.l3_off) & ~(uint64_t)15;
#pragma unroll
	for (int i = 0; i < kStrS; ++i) {
		const uint64_t src = a + 1024 * i + 16 * lane;
		const bool ok = live && src <= last_chunk;
		glds16_nt(ok ? reinterpret_cast<const void *>(src) : zero, lds_slot + 1024 * i);
	}
}

template <int kStrD>
__global__ __launch_bounds__(64) void stream_kernel(KParams p)
{
	extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
	uint8_t *ring = smem;
	uint32_t *so = reinterpret_cast<uint32_t *>(smem + kStrD * kStrSlot); // 4 * kStrWin outputs
	uint8_t *sv = reinterpret_cast<uint8_t *>(so + 4 * kStrWin);         // 4 * kStrWin verdicts
	const int lane = threadIdx.x & 63, g = lane >> 4, gl = lane & 15;
	const uint32_t flags = p.flags;
	const bool raw = flags & CGCK_RAW;
	const int len = (int)p.ip_len;
	const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)ring);
	const uint8_t *zero = (const uint8_t *)p.zero + (blockIdx.x & 63) * 64;
	const uint64_t base = reinterpret_cast<uint64_t>(p.base) + p.l3_off;
	const uint64_t last_chunk = (base + (p.n - 1) * p.stride + p.ip_len - 1) & ~(uint64_t)15;

	// Windows of kStrWin steps (4 kStrWin packets), grid-interleaved: wave b
	// takes windows b, b + G, ... so the grid sweeps one region of the batch
	// at a time (a contiguous range per wave measured 73-77 %; the
	// interleaved DMA sweep alone reads near the HBM peak, lpd_kernel).
	const uint64_t NW = (p.n + 4 * kStrWin - 1) / (4 * kStrWin);
	for (uint64_t win = blockIdx.x; win < NW; win += gridDim.x) {
		const uint64_t r0 = win * 4 * kStrWin;
		const uint64_t r1 = r0 + 4 * kStrWin < p.n ? r0 + 4 * kStrWin : p.n;
		const uint64_t nsteps = (r1 - r0 + 3) / 4;
		const uint64_t w0 = 0;
		const uint64_t wn = nsteps;
#pragma unroll
		for (int d = 0; d < kStrD - 1; ++d)
			str_issue(p, r0 + 4 * (w0 + d), (uint64_t)d < wn, last_chunk, zero, lds0 + d * kStrSlot);
		for (uint64_t j = 0; j < wn; ++j) {
			const uint32_t slot = (uint32_t)(j % kStrD);
			str_issue(p, r0 + 4 * (w0 + j + kStrD - 1), j + kStrD - 1 < wn, last_chunk, zero,
				  lds0 + (uint32_t)((j + kStrD - 1) % kStrD) * kStrSlot);
			asm volatile("s_waitcnt vmcnt(%0)" ::"i"((kStrD - 1) * kStrS) : "memory");
			__builtin_amdgcn_s_barrier();
			if (p.contig == 3) // $CGCK_STR_NOCONS: the DMA pipeline alone (A/B)
				continue;

			const uint64_t first = r0 + 4 * (w0 + j);
			const uint64_t a_reg = (base + first * p.stride) & ~(uint64_t)15;
			const uint64_t pk = first + g;
			const int o = (int)(base + pk * p.stride - a_reg); // packet g's byte offset in the slot
			const int q = o & 15, c0 = o >> 4;
			const int nch = (q + len + 15) >> 4;
			const uint8_t *sl = ring + slot * kStrSlot;
			uint4 w[kStrS];
#pragma unroll
			for (int s = 0; s < kStrS; ++s) {
				const int c = c0 + 16 * s + gl;
				w[s] = *reinterpret_cast<const uint4 *>(sl + 16 * (c < kStrS * 64 ? c : kStrS * 64 - 1));
			}
			// header words (same address for the group's lanes: broadcast);
			// packets are dword aligned, so these are dword loads
			const uint32_t *hw = reinterpret_cast<const uint32_t *>(sl + o);
			const uint32_t h0 = hw[0], h1 = hw[1], h2 = hw[2], h3 = hw[3], h4 = hw[4];
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // also: this slot is refilled next step

			uint32_t body = 0;
#pragma unroll
			for (int s = 0; s < kStrS; ++s)
				body = 16 * s + gl < nch ? sum4(w[s], body) : body;
			// bytes of the first chunk before the packet and of the last after it
			uint32_t corr = 0;
			if (gl == 0 && q != 0)
				corr = msum(w[0], 0, 0, q, 0);
			const int e = q + len - 16 * (nch - 1);
#pragma unroll
			for (int s = 0; s < kStrS; ++s)
				if (16 * s + gl == nch - 1 && e != 16)
					corr = fold16(corr) + fold16(msum(w[s], 0, e, 16, 0));
			uint32_t tot = fold16(body) + (0xffffu - fold16(corr));
			tot = fold16(gsum<16>(tot));

			if (gl == 0) {
				const uint32_t hd = h0 & 15;
				const int hl = (int)hd * 4;
				const uint32_t proto = (h2 >> 8) & 0xffu;
				uint32_t lo = 0, hi = 0, verdict = 0;
				if (raw) {
					lo = finish(tot);
				} else if (len < hl) {
					verdict = CGCK_BAD_LEN;
				} else {
					uint32_t ip = hsum(h4, hsum(h3, hsum(h2, hsum(h1, hsum(h0, 0)))));
					if (hd != 5) {
						ip = 0;
						for (uint32_t i = 0; i < hd; ++i)
							ip = hsum(hw[i], ip);
					}
					const uint32_t IPs = fold16(ip);
					if (flags & CGCK_IP)
						lo = finish(IPs);
					if (flags & CGCK_L4) {
						uint32_t L = ocsub(tot, IPs);
						if (!(flags & CGCK_L4_NOPSEUDO))
							L = fold16(L + fold16(hsum(h4, hsum(h3, 0))) + (proto << 8) +
								   bswap16((uint32_t)(len - hl) & 0xffffu));
						hi = finish(L);
					}
				}
				so[4 * j + g] = lo | (hi << 16);
				sv[4 * j + g] = (uint8_t)verdict;
			}
		}
		// window end: retire every DMA, then write the window's outputs
		asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
		__builtin_amdgcn_s_barrier();
		const uint64_t b = r0;
		const uint64_t cnt = r1 - r0;
		for (uint64_t i = lane; i < cnt; i += 64) {
			if (p.out)
				gbl(p.out)[b + i] = so[i];
			if (p.verdict)
				gbl(p.verdict)[b + i] = sv[i];
		}
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // so/sv are rewritten next window
	}
}

// ---------------------------------------------------------------------------
// Loader/consumer form: one wave per workgroup only moves bytes, three waves
// only compute (MI355X_MICROARCH.md 'ldsdma-fill': a dedicated LDS-DMA
// loader wave per CU streams at 6.4-6.8 TB/s beside its consumers).
// A phase is 3 steps (12 packets); the ring holds kLcPh phases (3 slots
// each).  Per phase: the loader waits (counted vmcnt) for phase ph, all four
// waves pass barrier ph, the loader refills the slots of phase ph-1 (which
// the consumers finished, lgkmcnt(0), before that barrier) with phase
// ph+kLcPh-1, and consumer c reduces step 3ph+c.  Consumers store their
// outputs directly: their stores count only in their own vmcnt.
// ---------------------------------------------------------------------------

template <int kLcPh>
__device__ __forceinline__ void lc_issue_phase(const KParams &p, uint64_t r0, uint64_t r1, uint64_t ph,
					       uint64_t last_chunk, const uint8_t *zero, uint32_t lds0)
{
	const uint32_t grp = (uint32_t)(ph % kLcPh) * 3;
#pragma unroll
	for (int c = 0; c < 3; ++c) {
		const uint64_t first = r0 + 4 * (3 * ph + c);
		str_issue(p, first, first < r1, last_chunk, zero, lds0 + (grp + c) * kStrSlot);
	}
}

__device__ __forceinline__ void str_consume(const KParams &p, const uint8_t *sl, uint64_t first, uint64_t r1,
					    uint64_t base)
{
	const int lane = threadIdx.x & 63, g = lane >> 4, gl = lane & 15;
	const uint32_t flags = p.flags;
	const bool raw = flags & CGCK_RAW;
	const int len = (int)p.ip_len;
	const uint64_t a_reg = (base + first * p.stride) & ~(uint64_t)15;
	const uint64_t pk = first + g;
	const int o = (int)(base + pk * p.stride - a_reg);
	const int q = o & 15, c0 = o >> 4;
	const int nch = (q + len + 15) >> 4;
	uint4 w[kStrS];
#pragma unroll
	for (int s = 0; s < kStrS; ++s) {
		const int c = c0 + 16 * s + gl;
		w[s] = *reinterpret_cast<const uint4 *>(sl + 16 * (c < kStrS * 64 ? c : kStrS * 64 - 1));
	}
	const uint32_t *hw = reinterpret_cast<const uint32_t *>(sl + o);
	const uint32_t h0 = hw[0], h1 = hw[1], h2 = hw[2], h3 = hw[3], h4 = hw[4];
	uint32_t body = 0;
#pragma unroll
	for (int s = 0; s < kStrS; ++s)
		body = 16 * s + gl < nch ? sum4(w[s], body) : body;
	uint32_t corr = 0;
	if (gl == 0 && q != 0)
		corr = msum(w[0], 0, 0, q, 0);
	const int e = q + len - 16 * (nch - 1);
#pragma unroll
	for (int s = 0; s < kStrS; ++s)
		if (16 * s + gl == nch - 1 && e != 16)
			corr = fold16(corr) + fold16(msum(w[s], 0, e, 16, 0));
	uint32_t tot = fold16(body) + (0xffffu - fold16(corr));
	tot = fold16(gsum<16>(tot));
	if (gl != 0 || pk >= r1)
		return;
	const uint32_t hd = h0 & 15;
	const int hl = (int)hd * 4;
	const uint32_t proto = (h2 >> 8) & 0xffu;
	uint32_t lo = 0, hi = 0, verdict = 0;
	if (raw) {
		lo = finish(tot);
	} else if (len < hl) {
		verdict = CGCK_BAD_LEN;
	} else {
		uint32_t ip = hsum(h4, hsum(h3, hsum(h2, hsum(h1, hsum(h0, 0)))));
		if (hd != 5) {
			ip = 0;
			for (uint32_t i = 0; i < hd; ++i)
				ip = hsum(hw[i], ip);
		}
		const uint32_t IPs = fold16(ip);
		if (flags & CGCK_IP)
			lo = finish(IPs);
		if (flags & CGCK_L4) {
			uint32_t L = ocsub(tot, IPs);
			if (!(flags & CGCK_L4_NOPSEUDO))
				L = fold16(L + fold16(hsum(h4, hsum(h3, 0))) + (proto << 8) +
					   bswap16((uint32_t)(len - hl) & 0xffffu));
			hi = finish(L);
		}
	}
	if (p.out)
		gbl(p.out)[pk] = lo | (hi << 16);
	if (p.verdict)
		gbl(p.verdict)[pk] = (uint8_t)verdict;
}

template <int kLcPh> // phases in the ring (3 slots of 6 KiB each)
__global__ __launch_bounds__(256) void stream_lc_kernel(KParams p)
{
	extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
	const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem);
	const uint8_t *zero = (const uint8_t *)p.zero + (blockIdx.x & 63) * 64;
	const uint64_t base = reinterpret_cast<uint64_t>(p.base) + p.l3_off;
	const uint64_t last_chunk = (base + (p.n - 1) * p.stride + p.ip_len - 1) & ~(uint64_t)15;
	// contiguous packet range of this workgroup, a multiple of 12 packets
	const uint64_t nb = gridDim.x;
	const uint64_t per = (((p.n + nb - 1) / nb) + 11) / 12 * 12;
	const uint64_t r0 = (uint64_t)blockIdx.x * per;
	const uint64_t r1 = r0 + per < p.n ? r0 + per : p.n;
	if (r0 >= r1)
		return; // uniform across the workgroup
	const uint64_t nph = (r1 - r0 + 11) / 12;

	if (wave == 0) {
#pragma unroll
		for (int d = 0; d < kLcPh - 1; ++d)
			lc_issue_phase<kLcPh>(p, r0, r1, d, last_chunk, zero, lds0);
		for (uint64_t ph = 0; ph < nph; ++ph) {
			// phase ph landed: phases ph+1 .. ph+kLcPh-2 may stay in flight
			asm volatile("s_waitcnt vmcnt(%0)" ::"i"((kLcPh - 2) * 3 * kStrS) : "memory");
			__builtin_amdgcn_s_barrier();
			lc_issue_phase<kLcPh>(p, r0, r1, ph + kLcPh - 1, last_chunk, zero, lds0);
		}
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	} else {
		const int c = wave - 1;
		for (uint64_t ph = 0; ph < nph; ++ph) {
			__builtin_amdgcn_s_barrier();
			const uint64_t first = r0 + 4 * (3 * ph + c);
			if (first < r1)
				str_consume(p, smem + ((uint32_t)(ph % kLcPh) * 3 + c) * kStrSlot, first, r1, base);
			// this phase's slots are refilled after the next barrier
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
		}
	}
}

bool stream_ok(const KParams &p)
{
	const uint32_t fl = p.flags;
	const bool flags_ok = fl == CGCK_RAW || (fl && !(fl & ~(uint32_t)(CGCK_IP | CGCK_L4 | CGCK_L4_NOPSEUDO)));
	return !p.desc && p.n > 0 && flags_ok && !p.bad && p.ip_len >= 20 && p.ip_len <= 1520 && p.stride <= 1520 &&
	       ((reinterpret_cast<uintptr_t>(p.base) | p.stride | p.l3_off) & 3) == 0;
}

hipError_t launch_stream(const KParams &p, int num_cus, hipStream_t st)
{
	static const int wpc = [] { // $CGCK_STR_WPC: waves per CU (A/B runs)
		const char *e = CGCK_ENV("CGCK_STR_WPC");
		return e && atoi(e) > 0 ? atoi(e) : 8;
	}();
	static const bool lc = [] { // $CGCK_STR_LC=1: the loader/consumer form
		const char *e = CGCK_ENV("CGCK_STR_LC");
		return e && *e == '1';
	}();
	if (lc) {
		static const int ph = [] { // $CGCK_STR_LCPH: ring phases 3 or 4 (vmcnt counts <= 63)
			const char *e = CGCK_ENV("CGCK_STR_LCPH");
			return e && atoi(e) == 3 ? 3 : 4;
		}();
		const uint64_t want = (p.n + 12 * 16 - 1) / (12 * 16); // >= 16 phases per workgroup
		const uint64_t cap = (uint64_t)num_cus * 2; // 54 / 72 KiB rings: 2 per CU
		const dim3 g((unsigned)(want < cap ? (want ? want : 1) : cap));
		if (ph == 3)
			hipLaunchKernelGGL(stream_lc_kernel<3>, g, dim3(256), 3 * 3 * kStrSlot, st, p);
		else
			hipLaunchKernelGGL(stream_lc_kernel<4>, g, dim3(256), 4 * 3 * kStrSlot, st, p);
		return hipGetLastError();
	}
	static const int ring = [] { // $CGCK_STR_RING: ring slots (A/B runs)
		const char *e = CGCK_ENV("CGCK_STR_RING");
		return e && atoi(e) >= 2 && atoi(e) <= 4 ? atoi(e) : 3;
	}();
	static const bool nocons = CGCK_ENV("CGCK_STR_NOCONS") != nullptr;
	KParams q = p;
	if (nocons)
		q.contig = 3;
	const uint64_t waves = (uint64_t)num_cus * wpc;
	const uint64_t want = (p.n + 63) / 64; // at least 16 steps per wave
	const dim3 g((unsigned)(want < waves ? (want ? want : 1) : waves));
	const size_t lds = ring * kStrSlot + 4 * kStrWin * 4 + 4 * kStrWin;
	if (ring == 2)
		hipLaunchKernelGGL(stream_kernel<2>, g, dim3(64), lds, st, q);
	else if (ring == 4)
		hipLaunchKernelGGL(stream_kernel<4>, g, dim3(64), lds, st, q);
	else
		hipLaunchKernelGGL(stream_kernel<3>, g, dim3(64), lds, st, q);
	return hipGetLastError();
}

} // namespace cgck
