// cgck_dense.hip — dense strided batches of large frames (the 1500 B config)
// streamed through LDS by DMA: dstr_kernel.
//
// What round 2 measured first (profiles/r02/dma/str*, lpd/): the LDS-DMA
// read alone reaches 88 % of 8 TB/s once the grid sweeps one window of the
// batch, against the register-load ceiling (78-81 %) the group kernel sits
// on, but the first stream kernel (cgck_stream.hip, lab) lost that with its
// consumer (78.8 % vs group 81.7 %).  Its pipeline drained at every window
// end (vmcnt(0) before a per-window output flush, then a fresh prologue),
// and its reduce ran the chunk corrections and the header in exec-masked
// branches.  This kernel keeps lpd_kernel's structure, which does pay at
// 64 B (cgck_lane.hip):
//
//  * A step = 4 consecutive frames: the chunks from the first frame's
//    16-byte-aligned start to the fourth frame's last chunk (<= 6 KiB when
//    stride, ip_len <= 1520), moved by 6 contiguous 1 KiB
//    global_load_lds_dwordx4 ... nt into a ring of D slots of the wave (one
//    wave per workgroup).  Lanes past the step's last chunk read the zero
//    line, so the only bytes read twice are one shared chunk per step.  A
//    step's slot is refilled as soon as its bytes are in registers, before
//    the reduce, so D steps are in flight through the arithmetic too.
//  * Steps come in chunks of C, chunks grid-interleaved (wave b takes chunks
//    b, b + G, ...): the grid sweeps one window of the batch.  The ring runs
//    across chunk boundaries without a drain: a chunk's 4C outputs are
//    staged in LDS and leave as ONE 16-byte store per lane (sc1) while the
//    next steps' DMA is in flight; the counted vmcnt for step j includes that
//    store when it was issued after step j's DMA.
//  * The reduce is branch-free per lane: lane (g = lane / 16, gl) sums region
//    chunks c0_g + 16 s + gl, s = 0..5, of frame g (chunks past the frame
//    select 0), and the group's lane 0 subtracts the bytes of its first chunk
//    before the frame (dword-aligned frames: whole dwords) and of its last
//    chunk after it (read once more from LDS as a broadcast).  The header
//    words are broadcast reads; every lane computes the frame's result (the
//    cost is per wave either way) and lane 0 of the group stages it.
//
// Scope (dstr_ok): strided batches, base / stride / l3_off multiples of 4,
// 20 <= ip_len <= 1520, stride <= 1520, flags RAW or any of IP / L4 /
// L4_NOPSEUDO (no field zeroing, verify or in-place store), an output array
// (16-byte aligned), optional verdicts (BAD_LEN only, with these flags) and
// no bad counters.  Everything else takes cgck_group.hip.
// Arithmetic: subr.c:127-223 as restated in cgck_device.h (one's-complement
// sums of 16-bit words in any order, folded; reduce's 0 -> 0xFFFF).
#include "cgck_device.h"

#include <stdlib.h>

namespace cgck {

constexpr int kDsS = 6;                     // DMA instructions (KiB) per step
constexpr uint32_t kDsSlot = kDsS * 1024;   // bytes per ring slot
constexpr int kDsChunks = kDsS * 64;        // 16-byte chunks per slot
// Every chunk a lane of the reducing wave reads lies in its slot, so the
// reads need no clamp: frame g of a step starts at most 15 + 3 * 1520 bytes
// into the slot (dstr_ok: stride <= 1520), and a lane reads up to 95 chunks
// past the frame's first (16 s + gl).  (Unclamped: 1.004 of the clamped
// reads in one process, twice, bit-exact; profiles/r04/dstr_ab/.)
static_assert(((15 + 3 * 1520) >> 4) + 16 * (kDsS - 1) + 15 < kDsChunks, "a reducing lane's chunk lies in its slot");

template <int D, int C, bool W, int F>
__global__ __launch_bounds__(128) void dstr_kernel(KParams p)
{
	extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
	const int lane = threadIdx.x & 63, g = lane >> 4, gl = lane & 15;
	const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const uint32_t flags = p.flags;
	const bool raw = flags & CGCK_RAW;
	const int len = (int)p.ip_len;
	const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem);
	// staged outputs of a chunk (W: the sums of 2 chunks, 2 words a frame)
	uint32_t *so = reinterpret_cast<uint32_t *>(smem + D * kDsSlot);
	const uint8_t *zero = (const uint8_t *)p.zero + (blockIdx.x & 63) * 64;
	const uint64_t base = reinterpret_cast<uint64_t>(p.base) + p.l3_off;
	const uint64_t n = p.n, stride = p.stride;
	// Super-chunks of SC frames, grid-interleaved: the first 4C are wave 0's
	// C steps, the last F the writer wave's (W, F > 0: read by register loads
	// while it waits for wave 0's chunk, so more bytes are in flight per CU
	// than the LDS ring holds).
	constexpr uint32_t SC = 4 * C + F;
	const uint64_t NC = (n + SC - 1) / SC, G = gridDim.x, b = blockIdx.x;
	if (b >= NC)
		return;
	const uint32_t nsteps = (uint32_t)((NC - b + G - 1) / G * C);
	const uint32_t mode = p.contig; // lab A/B modes (launch_dstr); 0 in the product
	auto cfirst = [&](uint32_t k) { return (b + (uint64_t)k * G) * SC; }; // chunk k's first frame

	// a frame's result from its folded sums (tot over the frame, ip over the
	// header, ps over src/dst), ip_hl and ip_p: result() of cgck_group.hip
	auto fin = [&](uint32_t tot, uint32_t ip, uint32_t ps, uint32_t hd, uint32_t proto) {
		const int hl = (int)hd * 4;
		uint32_t lo = 0, hi = 0;
		if (raw) {
			lo = finish(tot);
		} else if (len >= hl) { // else BAD_LEN: 0 | 0 << 16, as the group kernel
			if (flags & CGCK_IP)
				lo = finish(ip);
			if (flags & CGCK_L4) {
				uint32_t L = ocsub(tot, ip);
				if (!(flags & CGCK_L4_NOPSEUDO))
					L = fold16(L + ps + (proto << 8) + bswap16((uint32_t)(len - hl) & 0xffffu));
				hi = finish(L);
			}
		}
		return lo | (hi << 16);
	};

	// the outputs of chunk k (its 4C frames, staged at sb) to global memory
	auto flush = [&](uint32_t k, const uint32_t *sb) {
		const uint64_t first = cfirst(k);
		if (first + 4 * C <= n) {
			if (lane < C) { // one 16-byte store per lane
				const uint4 v4 = reinterpret_cast<const uint4 *>(sb)[lane];
				bstore16<kSc1>(out_rsrc(p.out + first, 16 * C), 16 * lane, u32x4_t{v4.x, v4.y, v4.z, v4.w});
			}
		} else { // the batch's last, partial chunk: per-frame stores
			for (int i = lane; i < 4 * C; i += 64)
				if (first + i < n)
					gbl(p.out)[first + i] = sb[i];
		}
	};

	// A frame read into registers by its 16 lanes (chunks c0 + 16 s + gl,
	// clamped): the same sums as wave 0 takes from LDS; lane 0 stores it.
	auto reg_frame = [&](uint64_t f, uint64_t a, int nch, const uint4 (&w)[kDsS]) __attribute__((always_inline)) {
		const int q = (int)(a & 15);
		uint32_t body = 0;
		uint4 tw = make_uint4(0, 0, 0, 0); // the frame's last chunk, in the lane holding it
		bool ht = false;
#pragma unroll
		for (int s2 = 0; s2 < kDsS; ++s2) {
			const int c = 16 * s2 + gl;
			body += c < nch ? sum4(w[s2], 0u) : 0u;
			const bool t = c == nch - 1;
			// opaque masks: a select chain over array elements would be turned
			// into a dynamically indexed (scratch) load
			const uint32_t mt = opaque(t ? ~0u : 0u);
			tw = make_uint4(pick(mt, w[s2].x, tw.x), pick(mt, w[s2].y, tw.y), pick(mt, w[s2].z, tw.z),
					pick(mt, w[s2].w, tw.w));
			ht = ht || t;
		}
		uint32_t corr = 0;
		if (gl == 0) { // the q bytes (whole dwords) before the frame
			corr = hsum(q >= 4 ? w[0].x : 0u, 0);
			corr = hsum(q >= 8 ? w[0].y : 0u, corr);
			corr = hsum(q >= 12 ? w[0].z : 0u, corr);
		}
		if (ht) { // the bytes of the last chunk after the frame
			const int e = q + len - 16 * (nch - 1);
			if ((len & 3) == 0) {
				corr = hsum(e <= 4 ? tw.y : 0u, corr);
				corr = hsum(e <= 8 ? tw.z : 0u, corr);
				corr = hsum(e <= 12 ? tw.w : 0u, corr);
			} else {
				corr = msum(tw, 0, e, 16, corr);
			}
		}
		uint32_t tot = fold16(body) + (0xffffu - fold16(corr));
		tot = fold16(gsum<16>(tot));
		// header dwords: chunk c0 (this lane) and c0 + 1 (lane gl + 1, DPP row_shl:1)
		const uint32_t n0 = __builtin_amdgcn_mov_dpp(w[0].x, 0x101, 0xF, 0xF, false);
		const uint32_t n1 = __builtin_amdgcn_mov_dpp(w[0].y, 0x101, 0xF, 0xF, false);
		const uint32_t n2 = __builtin_amdgcn_mov_dpp(w[0].z, 0x101, 0xF, 0xF, false);
		const uint32_t n3 = __builtin_amdgcn_mov_dpp(w[0].w, 0x101, 0xF, 0xF, false);
		const uint32_t d[8] = {w[0].x, w[0].y, w[0].z, w[0].w, n0, n1, n2, n3};
		const int q4 = q >> 2;
		const uint32_t m0 = opaque(q4 == 0 ? ~0u : 0u), m1 = opaque(q4 == 1 ? ~0u : 0u),
			       m2 = opaque(q4 == 2 ? ~0u : 0u);
		uint32_t h[5];
#pragma unroll
		for (int i = 0; i < 5; ++i)
			h[i] = pick(m0, d[i], pick(m1, d[i + 1], pick(m2, d[i + 2], d[i + 3])));
		const uint32_t hd = h[0] & 15;
		uint32_t ip = hsum(h[4], hsum(h[3], hsum(h[2], hsum(h[1], hsum(h[0], 0)))));
		if (gl == 0 && f < n) {
			if (hd != 5) { // options or a short header (rare): from global memory
				ip = 0;
				for (uint32_t i = 0; i < hd; ++i)
					ip = hsum(*gbl_at<const uint32_t>(a + 4 * i), ip);
			}
			const uint32_t r = fin(tot, fold16(ip), fold16(hsum(h[4], hsum(h[3], 0))), hd, (h[2] >> 8) & 0xffu);
			gbl(p.out)[f] = r;
			if (p.verdict)
				gbl(p.verdict)[f] = (uint8_t)(!raw && len < (int)hd * 4 ? CGCK_BAD_LEN : 0);
		}
	};

	if (W && wave == 1) {
		// The writer wave finishes and stores each chunk's frames, a lane per
		// frame, from the sums wave 0 staged: no store sits in the reducing
		// wave's vmcnt, where (in order) it would hold the wait for every
		// later step's DMA, and the per-frame finish leaves its VALU.  One
		// barrier per chunk (the staging is double-buffered: wave 0 refills a
		// buffer only after the next chunk's barrier, which this wave reaches
		// once it has read it); lab mode 6 adds wave 0's per-step barrier.
		for (uint32_t j = 0; j < nsteps; ++j) {
			if (mode == 6)
				wg_barrier();
			if ((j + 1) % C == 0) {
				const uint32_t k = j / C;
				// the chunk's F register frames: loads in flight across the wait
				uint4 rw[F > 0 ? F / 4 : 1][kDsS];
				uint64_t ra[F > 0 ? F / 4 : 1];
				int rn[F > 0 ? F / 4 : 1];
#pragma unroll
				for (int u = 0; u < F / 4; ++u) {
					const uint64_t f = cfirst(k) + 4 * C + 4 * u + g;
					ra[u] = base + (f < n ? f : 0) * stride;
					rn[u] = f < n ? (int)(((ra[u] & 15) + len + 15) >> 4) : 0;
					const uint4 *c0 = reinterpret_cast<const uint4 *>(ra[u] & ~(uint64_t)15);
#pragma unroll
					for (int s2 = 0; s2 < kDsS; ++s2)
						rw[u][s2] = ldc<true>(c0, 16 * s2 + gl, rn[u], p.zero);
				}
				wg_barrier(); // chunk j / C staged
				const uint32_t *sb = so + (k & 1) * 8 * C;
				const uint64_t first = cfirst(k);
				for (int i = lane; i < 4 * C; i += 64) {
					const uint32_t v0 = sb[i], v1 = sb[4 * C + i];
					const uint32_t hd = (v1 >> 16) & 15u;
					const uint32_t r = fin(v0 & 0xffffu, v0 >> 16, v1 & 0xffffu, hd, v1 >> 24);
					if (p.verdict && first + i < n) // BAD_LEN, as the group kernel
						gbl(p.verdict)[first + i] = (uint8_t)(!raw && len < (int)hd * 4 ? CGCK_BAD_LEN : 0);
					if (first + 4 * C <= n)
						bstore4<kSc1>(out_rsrc(p.out + first, 16 * C), 4 * i, r);
					else if (first + i < n)
						gbl(p.out)[first + i] = r;
				}
#pragma unroll
				for (int u = 0; u < F / 4; ++u)
					reg_frame(cfirst(k) + 4 * C + 4 * u + g, ra[u], rn[u], rw[u]);
			}
		}
		return;
	}

	auto sfirst = [&](uint32_t j) { return cfirst(j / C) + 4 * (j % C); }; // step j's first frame
	auto issue = [&](uint32_t j) { // step j of this wave into slot j % D
		const uint64_t f0 = sfirst(j);
		const bool live = j < nsteps && f0 < n;
		const uint64_t fl = f0 + 3 < n ? f0 + 3 : n - 1;
		const uint64_t a = (base + f0 * stride) & ~(uint64_t)15;
		const uint64_t e = (base + fl * stride + len - 1) & ~(uint64_t)15; // the step's last chunk
		const uint32_t slot = lds0 + (j % D) * kDsSlot;
#pragma unroll
		for (int i = 0; i < kDsS; ++i) {
			const uint64_t s0 = a + 1024 * i, src = s0 + 16 * lane;
			if (live && s0 + 1008 <= e) // the whole KiB lies in the step (wave-uniform)
				glds16_nt(reinterpret_cast<const void *>(src), slot + 1024 * i);
			else
				glds16_nt(live && src <= e ? reinterpret_cast<const void *>(src) : zero, slot + 1024 * i);
		}
	};
#pragma unroll
	for (int d = 0; d < D; ++d)
		issue(d);
	for (uint32_t j = 0; j < nsteps; ++j) {
		// Wait for step j's DMA.  Issued after it: the D - 1 later steps' DMA
		// and (without the writer wave) the last chunk flush's store when it
		// came after step j's DMA.
		if (!W && j >= (uint32_t)C && (j % C) <= (uint32_t)(D - 1))
			asm volatile("s_waitcnt vmcnt(%0)" ::"i"(kDsS * (D - 1) + 1) : "memory");
		else
			asm volatile("s_waitcnt vmcnt(%0)" ::"i"(kDsS * (D - 1)) : "memory");
		// The covering vmcnt alone orders this wave's own ds_reads behind its
		// LDS-DMA (MI355X_MICROARCH.md: a barrier is needed only for other
		// waves' reads), so no barrier per step.
		if (!W || mode == 6)
			wg_barrier();
		uint32_t *sc = so + (W ? ((j / C) & 1) * 8 * C : 0); // this chunk's staging
		if (mode == 3) { // lab: the DMA pipeline alone
			issue(j + D);
		} else {
			const uint64_t f0 = sfirst(j);
			const uint64_t a = (base + f0 * stride) & ~(uint64_t)15;
			const int o = (int)(base + (f0 + g) * stride - a); // frame g's byte offset in the slot
			const int q = o & 15, c0 = o >> 4;
			const int nch = (q + len + 15) >> 4;
			const uint8_t *sl = smem + (j % D) * kDsSlot;
			uint4 w[kDsS];
#pragma unroll
			for (int s = 0; s < kDsS; ++s) {
				const int c = c0 + 16 * s + gl;
				w[s] = *reinterpret_cast<const uint4 *>(sl + 16 * c);
			}
#if CGCK_DSTR_REGHDR
			// (lab A/B) only the six chunk reads before the refill: the last
			// chunk is the register of the lane holding it, the header dwords
			// come from w[0] of this lane and the next (DPP row_shl:1)
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
			issue(j + D);
			uint4 wt = make_uint4(0, 0, 0, 0);
			bool ht = false;
#pragma unroll
			for (int s = 0; s < kDsS; ++s) {
				const bool t = 16 * s + gl == nch - 1;
				const uint32_t mt = opaque(t ? ~0u : 0u);
				wt = make_uint4(pick(mt, w[s].x, wt.x), pick(mt, w[s].y, wt.y), pick(mt, w[s].z, wt.z),
						pick(mt, w[s].w, wt.w));
				ht = ht || t;
			}
			const uint32_t n0 = __builtin_amdgcn_mov_dpp(w[0].x, 0x101, 0xF, 0xF, false);
			const uint32_t n1 = __builtin_amdgcn_mov_dpp(w[0].y, 0x101, 0xF, 0xF, false);
			const uint32_t n2 = __builtin_amdgcn_mov_dpp(w[0].z, 0x101, 0xF, 0xF, false);
			const uint32_t n3 = __builtin_amdgcn_mov_dpp(w[0].w, 0x101, 0xF, 0xF, false);
			const uint32_t dd[8] = {w[0].x, w[0].y, w[0].z, w[0].w, n0, n1, n2, n3};
			const int q4 = q >> 2;
			const uint32_t m0 = opaque(q4 == 0 ? ~0u : 0u), m1 = opaque(q4 == 1 ? ~0u : 0u),
				       m2 = opaque(q4 == 2 ? ~0u : 0u);
			uint32_t hh[5];
#pragma unroll
			for (int i = 0; i < 5; ++i)
				hh[i] = pick(m0, dd[i], pick(m1, dd[i + 1], pick(m2, dd[i + 2], dd[i + 3])));
			const uint32_t h2 = hh[2], h3 = hh[3], h4 = hh[4];
			const uint32_t hd = hh[0] & 15;
			uint32_t ip = hsum(h4, hsum(h3, hsum(h2, hsum(hh[1], hsum(hh[0], 0)))));
			if (gl == 0 && hd != 5 && f0 + g < n) { // options or a short header (rare): global memory
				const uint64_t fa = base + (f0 + g) * stride;
				ip = 0;
				for (uint32_t i = 0; i < hd; ++i)
					ip = hsum(*gbl_at<const uint32_t>(fa + 4 * i), ip);
			}
#else
			const uint4 wt = *reinterpret_cast<const uint4 *>(sl + 16 * (c0 + nch - 1)); // the last chunk
			const uint32_t *hw = reinterpret_cast<const uint32_t *>(sl + o);
			const uint32_t h0 = hw[0], h1 = hw[1], h2 = hw[2], h3 = hw[3], h4 = hw[4];
			const uint32_t hd = h0 & 15;
			uint32_t ip = hsum(h4, hsum(h3, hsum(h2, hsum(h1, hsum(h0, 0)))));
			if (hd != 5) { // options or a short header (exec-masked, rare)
				ip = 0;
				for (uint32_t i = 0; i < hd; ++i)
					ip = hsum(hw[i], ip);
			}
			// The slot's bytes are in registers: refill it now, so D steps stay
			// in flight while this one is reduced.
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
			issue(j + D);
#endif

			// independent per-chunk chains (no dependent v_dot2 wait states),
			// then the chunks inside the frame
			uint32_t cs[kDsS];
#pragma unroll
			for (int s = 0; s < kDsS; ++s)
				cs[s] = sum4(w[s], 0);
			uint32_t body = 0;
#pragma unroll
			for (int s = 0; s < kDsS; ++s)
				body += (len >= 1280 && s < 5) || 16 * s + gl < nch ? cs[s] : 0u;
			// group lane 0: the q bytes (whole dwords) of the first chunk before
			// the frame and the bytes of the last chunk after it
			uint32_t lead = hsum(q >= 4 ? w[0].x : 0u, 0);
			lead = hsum(q >= 8 ? w[0].y : 0u, lead);
			lead = hsum(q >= 12 ? w[0].z : 0u, lead);
			const int e = q + len - 16 * (nch - 1); // bytes of the last chunk in the frame
			uint32_t tail;
			if ((len & 3) == 0) { // whole dwords (kernel-uniform)
				tail = hsum(e <= 4 ? wt.y : 0u, 0);
				tail = hsum(e <= 8 ? wt.z : 0u, tail);
				tail = hsum(e <= 12 ? wt.w : 0u, tail);
			} else {
				tail = msum(wt, 0, e, 16, 0);
			}
#if CGCK_DSTR_REGHDR
			const uint32_t corr = (gl == 0 ? lead : 0u) + (ht ? tail : 0u);
#else
			const uint32_t corr = gl == 0 ? lead + tail : 0u;
#endif
			uint32_t tot = fold16(body) + (0xffffu - fold16(corr));
			tot = fold16(gsum<16>(tot));

			const uint32_t proto = (h2 >> 8) & 0xffu;
			const uint32_t ps = fold16(hsum(h4, hsum(h3, 0)));
			if (W) { // the writer wave finishes: stage the sums
				if (gl == 0) {
					sc[4 * (j % C) + g] = tot | (fold16(ip) << 16);
					sc[4 * C + 4 * (j % C) + g] = ps | (hd << 16) | (proto << 24);
				}
			} else if (gl == 0) {
				sc[4 * (j % C) + g] = fin(tot, fold16(ip), ps, hd, proto);
			}
		}
		if ((j + 1) % C == 0) {
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // the chunk's outputs are in LDS
			if (W)
				wg_barrier(); // hand the chunk to the writer wave
			else if (mode != 2) // lab mode 2: no output flush
				flush(j / C, sc);
		}
	}
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

bool dstr_ok(const KParams &p)
{
	const uint32_t fl = p.flags;
	const bool flags_ok = fl == CGCK_RAW || (fl && !(fl & ~(uint32_t)(CGCK_IP | CGCK_L4 | CGCK_L4_NOPSEUDO)));
	return !p.desc && p.n > 0 && p.n < (1ull << 34) && flags_ok && !p.bad && p.out &&
	       (reinterpret_cast<uintptr_t>(p.out) & 15) == 0 && p.ip_len >= 20 && p.ip_len <= 1520 &&
	       p.stride <= 1520 && ((reinterpret_cast<uintptr_t>(p.base) | p.stride | p.l3_off) & 3) == 0;
}

#if CGCK_LAB
static int env_int(const char *name, int dflt)
{
	const char *e = getenv(name);
	return e && *e ? atoi(e) : dflt;
}
#endif

hipError_t launch_dstr(const KParams &p, int num_cus, hipStream_t st)
{
	KParams q = p;
	q.contig = 0;
#if CGCK_LAB
	// $CGCK_DSTR_D (ring slots 2 | 3 | 4), $CGCK_DSTR_C (steps per chunk 8 |
	// 16 | 32), $CGCK_DSTR_W (1: the writer wave), $CGCK_DSTR_F (frames per
	// chunk the writer reads by register loads: 0 | 4 | 8), $CGCK_DSTR_WPC (workgroups
	// per CU), $CGCK_DSTR_MODE (2 no output flush, 3 the DMA alone; results
	// then undefined; 6 a barrier per step in both waves): A/B knobs of the
	// lab build, read once
	static const int D = env_int("CGCK_DSTR_D", 3), C = env_int("CGCK_DSTR_C", 16),
			 Wr = env_int("CGCK_DSTR_W", 1), wpc = env_int("CGCK_DSTR_WPC", 8),
			 Fr = env_int("CGCK_DSTR_F", 0);
	static const int mode = env_int("CGCK_DSTR_MODE", 0);
	q.contig = mode;
	const uint64_t NC = (p.n + 4 * C + Fr - 1) / (4 * C + Fr);
	const uint64_t waves = (uint64_t)num_cus * wpc;
	const dim3 g((unsigned)(NC < waves ? NC : waves));
#define CGCK_DSTR(DD, CC, WW, FF)                                                                       \
	if (D == DD && C == CC && (Wr == 1 || p.verdict) == WW && Fr == FF) {                           \
		CGCK_NOTE_KERNEL("dstr_kernel<%d, %d, %s, %d>", DD, CC, tf(WW), FF);                     \
		hipLaunchKernelGGL((dstr_kernel<DD, CC, WW, FF>), g, dim3((WW) ? 128 : 64),               \
				   (DD) * kDsSlot + ((WW) ? 64 : 16) * (CC), st, q);                        \
		return hipGetLastError();                                                               \
	}
	CGCK_DSTR(3, 16, true, 4) CGCK_DSTR(3, 16, true, 8) CGCK_DSTR(3, 32, true, 8) CGCK_DSTR(3, 32, true, 4)
	CGCK_DSTR(3, 32, true, 0) CGCK_DSTR(3, 8, true, 0) CGCK_DSTR(2, 32, true, 0) CGCK_DSTR(4, 16, true, 0)
	CGCK_DSTR(3, 16, false, 0) CGCK_DSTR(3, 32, false, 0) CGCK_DSTR(2, 32, false, 0)
#undef CGCK_DSTR
#else
	// 8 workgroups (a reducing wave + the writer wave) per CU: 19 KiB of LDS
	// each (three 6 KiB slots + two chunks of staged sums)
	const uint64_t NC = (p.n + 63) / 64;
	const uint64_t waves = (uint64_t)num_cus * 8;
	const dim3 g((unsigned)(NC < waves ? NC : waves));
#endif
	CGCK_NOTE_KERNEL("dstr_kernel<3, 16, true, 0>");
	hipLaunchKernelGGL((dstr_kernel<3, 16, true, 0>), g, dim3(128), 3 * kDsSlot + 64 * 16, st, q);
	return hipGetLastError();
}

} // namespace cgck
