// cgck_device.h — device-side helpers shared by the gfx950 checksum kernels.
//
// Arithmetic of con-gen's checksum unit (subr.c:119-223) restated for lanes:
// 16-bit halves summed into u32 partials (v_dot2_u32_u16), one's-complement
// folds, the reduce() finish with its 0 -> 0xFFFF rule (subr.c:150-154).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cgck_internal.h"

namespace cgck {

#define CGCK_GLOBAL __attribute__((address_space(1)))

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

// The same byte-range masks from one 16-bit mask per chunk (the group body's
// header zone, eat<>): bit b set when byte b of the chunk at packet-relative
// co lies in [r0, r1).  A dword's byte mask is its nibble spread by one
// multiply (bit j -> byte j), about half the VALU of four dmask() (tools/srvlat:
// the header zone was half of a one-packet server request).
__device__ __forceinline__ uint32_t cmask16(int co, int r0, int r1)
{
	const int s = min(max(r0 - co, 0), 16), e = min(max(r1 - co, 0), 16);
	return e > s ? ((1u << e) - 1u) & ~((1u << s) - 1u) : 0u;
}

__device__ __forceinline__ uint32_t nibmask(uint32_t m, int i)
{
	const uint32_t n = (m >> (4 * i)) & 15u;
	return ((n * 0x00204081u) & 0x01010101u) * 0xffu;
}

__device__ __forceinline__ uint32_t msum16(const uint4 &w, uint32_t m, uint32_t acc)
{
	acc = hsum(w.x & nibmask(m, 0), acc);
	acc = hsum(w.y & nibmask(m, 1), acc);
	acc = hsum(w.z & nibmask(m, 2), acc);
	acc = hsum(w.w & nibmask(m, 3), acc);
	return acc;
}

__device__ __forceinline__ void zero16(uint4 &w, uint32_t m)
{
	w.x &= ~nibmask(m, 0);
	w.y &= ~nibmask(m, 1);
	w.z &= ~nibmask(m, 2);
	w.w &= ~nibmask(m, 3);
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

__device__ __forceinline__ bool l4_nopseudo(uint32_t proto, uint32_t flags)
{
	return (flags & CGCK_L4_NOPSEUDO) || ((flags & kFlagL4Auto) && proto == 1);
}

__device__ __forceinline__ int l4_field(uint32_t proto, uint32_t flags)
{
	if (l4_nopseudo(proto, flags))
		return proto == 1 ? 2 : -1;
	return proto == 6 ? 16 : (proto == 17 ? 6 : -1);
}

// kFlagRx: which of the stack's verify calls a frame of `avail` bytes can
// see (cgck_internal.h), from its first header bytes.  Returns the meta word
// and sets *cover to the bytes to sum: min(ntohs(ip_len), avail), at least
// the header; 0 when the stack drops the frame before any checksum
// (ip_input.c:28-44, gbtcp/inet.c:282-306: 20 <= ip_hl * 4 <= len).  The L4
// value is asked for only when the frame holds ntohs(ip_len) bytes
// (ip_input.c:76, gbtcp/inet.c:314) and the segment its header
// (tcp_input.c:67, udp_usrreq.c:65, ip_icmp.c:177).
__device__ __forceinline__ uint32_t rx_meta(uint32_t avail, uint32_t b0, uint32_t tl_hi, uint32_t tl_lo,
					    uint32_t proto, uint32_t *cover)
{
	const uint32_t hl = (b0 & 15) * 4;
	if (avail < 20 || hl < 20 || hl > avail) {
		*cover = 0;
		return 0;
	}
	const uint32_t total = tl_hi << 8 | tl_lo;
	uint32_t cv = total < avail ? total : avail;
	*cover = cv < hl ? hl : cv;
	const uint32_t l4len = total >= hl ? total - hl : 0;
	const uint32_t need = proto == 6 ? 18 : proto == 17 ? 8 : proto == 1 ? 4 : 0xffffffffu;
	uint32_t m = kRxOkIp | (proto == 1 ? kRxIcmp : 0) | hl << 8 | l4len << 16;
	if (total >= hl && total <= avail && l4len >= need)
		m |= kRxOkL4;
	return m;
}

__device__ __forceinline__ void store16(uint8_t *p, uint32_t v)
{
	if ((reinterpret_cast<uintptr_t>(p) & 1) == 0) {
		*(CGCK_GLOBAL uint16_t *)p = (uint16_t)v;
	} else {
		((CGCK_GLOBAL uint8_t *)p)[0] = (uint8_t)v;
		((CGCK_GLOBAL uint8_t *)p)[1] = (uint8_t)(v >> 8);
	}
}

// Stores, or (SYS) system-coherent ones (sc0 sc1: written through to the
// memory they name, complete when visible there) — the burst server's
// outputs in host memory.
template <bool SYS>
__device__ __forceinline__ void st32p(CGCK_GLOBAL uint32_t *p, uint32_t v)
{
	if (SYS)
		__hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
	else
		*p = v;
}

template <bool SYS>
__device__ __forceinline__ void st8p(CGCK_GLOBAL uint8_t *p, uint8_t v)
{
	if (SYS)
		__hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
	else
		*p = v;
}

template <bool SYS>
__device__ __forceinline__ void store16p(uint8_t *p, uint32_t v)
{
	if (!SYS) {
		store16(p, v);
	} else if ((reinterpret_cast<uintptr_t>(p) & 1) == 0) {
		__hip_atomic_store((CGCK_GLOBAL uint16_t *)p, (uint16_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
	} else {
		__hip_atomic_store((CGCK_GLOBAL uint8_t *)p, (uint8_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
		__hip_atomic_store((CGCK_GLOBAL uint8_t *)p + 1, (uint8_t)(v >> 8), __ATOMIC_RELAXED,
				   __HIP_MEMORY_SCOPE_SYSTEM);
	}
}

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// Packet memory, descriptors and outputs are addressed through explicit
// GLOBAL (address space 1) pointers.  Pointers rebuilt from integer
// arithmetic are generic to the compiler, which then emits flat_* memory
// ops: those count against both vmcnt and lgkmcnt, return out of order and
// force every wait to vmcnt(0) lgkmcnt(0) — including a wait on each
// iteration's output store.  global_* ops keep precise, in-order counting.
template <class T>
__device__ __forceinline__ CGCK_GLOBAL T *gbl(T *p)
{
	return (CGCK_GLOBAL T *)p;
}

template <class T>
__device__ __forceinline__ CGCK_GLOBAL T *gbl_at(uint64_t a)
{
	return (CGCK_GLOBAL T *)a;
}

// Streaming chunk load; NT = nontemporal (read-once data, no cache retention).
// 16 bytes per lane from global memory into LDS by DMA (global_load_lds_dwordx4,
// nontemporal): lane l's bytes land at lds_dst + 16 l (lds_dst wave-uniform, in
// M0).  Inline asm, so the compiler counts none of it in vmcnt: every wait on
// it is explicit in the caller.
__device__ __forceinline__ void glds16_nt(const void *gsrc, uint32_t lds_dst)
{
	uint32_t keep;
	asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\t"
		     "s_mov_b32 m0, %0"
		     : "=&s"(keep)
		     : "v"(gsrc), "s"(lds_dst)
		     : "memory");
}

// Output stores with a cache policy, as compiler-visible buffer stores
// (raw_buffer_store with the gfx950 cache-policy operand: kSc1 = sc1, kNt =
// nt).  The compiler's hazard recognizer then places the wait state a store
// of more than 8 bytes needs before a VALU may overwrite its data VGPRs (an
// inline-asm store needed a hand-written "s_nop 1": a writer wave that reused
// the registers right away stored the next address over two dwords of the
// data), and its own waits see the stores.  The resource covers
// [base, base + bytes): `base` is wave-uniform; a store past `bytes` is
// dropped by the range check instead of landing anywhere.
constexpr int kSc1 = 16, kNt = 2, kDefaultPolicy = 0;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t out_rsrc(const void *base, uint32_t bytes)
{
	return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, (int)bytes, 0x00020000);
}
template <int POLICY>
__device__ __forceinline__ void bstore16(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4_t v)
{
	__builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, POLICY);
}
template <int POLICY>
__device__ __forceinline__ void bstore4(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t v)
{
	__builtin_amdgcn_raw_buffer_store_b32(v, r, (int)off, 0, POLICY);
}

// s_barrier that the optimizer cannot move memory operations across: the
// builtin alone carries no memory semantics, so LDS loads after it may be
// hoisted above it (a wave handing staged LDS data to another wave needs
// both sides ordered).
__device__ __forceinline__ void wg_barrier()
{
	asm volatile("s_barrier" ::: "memory");
}

// Write count u32 outputs staged in LDS (src) to global dst, threads t of nt
// cooperating.  CGCK_FLUSH_POLICY (A/B builds): 0 nontemporal u32 stores, 1 u32
// with sc1, 2 16-byte stores with sc1 (dst aligned up by a u32 head, u32
// tail), 3 16-byte nontemporal stores.  Stores through inline asm are
// invisible to the compiler's vmcnt accounting; since the counter retires in
// order, an extra store only makes its waits stricter.
#ifndef CGCK_FLUSH_POLICY
#define CGCK_FLUSH_POLICY 0
#endif
__device__ __forceinline__ void flush_u32(const uint32_t *src, uint32_t *dst, int count, int t, int nt)
{
#if CGCK_FLUSH_POLICY == 0
	for (int i = t; i < count; i += nt)
		__builtin_nontemporal_store(src[i], (CGCK_GLOBAL uint32_t *)dst + i);
#elif CGCK_FLUSH_POLICY == 1
	for (int i = t; i < count; i += nt)
		asm volatile("global_store_dword %0, %1, off sc1" ::"v"(dst + i), "v"(src[i]) : "memory");
#else
	int head = (int)(((16 - ((uintptr_t)dst & 15)) & 15) >> 2);
	head = head < count ? head : count;
	if (t < head)
		asm volatile("global_store_dword %0, %1, off sc1" ::"v"(dst + t), "v"(src[t]) : "memory");
	const int body = (count - head) >> 2;
	for (int i = t; i < body; i += nt) {
		const uint32_t *s4 = src + head + 4 * i;
		const u32x4_t v = {s4[0], s4[1], s4[2], s4[3]};
#if CGCK_FLUSH_POLICY == 3
		asm volatile("global_store_dwordx4 %0, %1, off nt\n\ts_nop 1" ::"v"(dst + head + 4 * i), "v"(v) : "memory");
#else
		asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(dst + head + 4 * i), "v"(v) : "memory");
#endif
	}
	for (int i = head + 4 * body + t; i < count; i += nt)
		asm volatile("global_store_dword %0, %1, off sc1" ::"v"(dst + i), "v"(src[i]) : "memory");
#endif
}

template <bool NT>
__device__ __forceinline__ uint4 ld(const uint4 *p)
{
	if (NT) {
		u32x4_t x = __builtin_nontemporal_load((const CGCK_GLOBAL u32x4_t *)p);
		return make_uint4(x[0], x[1], x[2], x[3]);
	}
	const u32x4_t x = *(const CGCK_GLOBAL u32x4_t *)p;
	return make_uint4(x[0], x[1], x[2], x[3]);
}

// Branch-free chunk load: chunk i of a run of nch chunks starting at c0;
// indices past the run re-read its last chunk (same cache line, no extra HBM
// traffic) and lanes without chunks read the context's zero chunk, so no
// load sits in an exec-masked branch and vmcnt counting stays precise.  The
// caller drops the contribution of indices >= nch.
template <bool NT>
__device__ __forceinline__ uint4 ldc(const uint4 *c0, int i, int nch, const void *zero)
{
	return ld<NT>(nch > 0 ? c0 + min(i, nch - 1) : reinterpret_cast<const uint4 *>(zero));
}

// Two 16-byte system-coherent loads (global_load ... sc0 sc1), waited for
// (inline asm: the compiler counts none of it, so the wait is inside): the
// burst server's block read, coherent with the host's stores whatever the L2
// holds, without a cache invalidate; whole-line requests like plain loads
// (relaxed 8-byte atomic loads leave as one fabric read each).
template <int N>
__device__ __forceinline__ void ld_sys16xN(const uint4 *const (&a)[N], uint4 (&v)[N]);

__device__ __forceinline__ void ld_sys16x2(const uint4 *p0, const uint4 *p1, uint4 &v0, uint4 &v1)
{
	u32x4_t a, b;
	asm volatile("global_load_dwordx4 %0, %2, off sc0 sc1\n\t"
		     "global_load_dwordx4 %1, %3, off sc0 sc1\n\t"
		     "s_waitcnt vmcnt(0)"
		     : "=&v"(a), "=&v"(b)
		     : "v"(p0), "v"(p1)
		     : "memory");
	v0 = make_uint4(a[0], a[1], a[2], a[3]);
	v1 = make_uint4(b[0], b[1], b[2], b[3]);
}

template <>
__device__ __forceinline__ void ld_sys16xN<2>(const uint4 *const (&a)[2], uint4 (&v)[2])
{
	ld_sys16x2(a[0], a[1], v[0], v[1]);
}

// Six at once (the 16-lane group body's chunks), one wait for all.
template <>
__device__ __forceinline__ void ld_sys16xN<6>(const uint4 *const (&a)[6], uint4 (&v)[6])
{
	u32x4_t r0, r1, r2, r3, r4, r5;
	asm volatile("global_load_dwordx4 %0, %6, off sc0 sc1\n\t"
		     "global_load_dwordx4 %1, %7, off sc0 sc1\n\t"
		     "global_load_dwordx4 %2, %8, off sc0 sc1\n\t"
		     "global_load_dwordx4 %3, %9, off sc0 sc1\n\t"
		     "global_load_dwordx4 %4, %10, off sc0 sc1\n\t"
		     "global_load_dwordx4 %5, %11, off sc0 sc1\n\t"
		     "s_waitcnt vmcnt(0)"
		     : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3), "=&v"(r4), "=&v"(r5)
		     : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5])
		     : "memory");
	v[0] = make_uint4(r0[0], r0[1], r0[2], r0[3]);
	v[1] = make_uint4(r1[0], r1[1], r1[2], r1[3]);
	v[2] = make_uint4(r2[0], r2[1], r2[2], r2[3]);
	v[3] = make_uint4(r3[0], r3[1], r3[2], r3[3]);
	v[4] = make_uint4(r4[0], r4[1], r4[2], r4[3]);
	v[5] = make_uint4(r5[0], r5[1], r5[2], r5[3]);
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

// Block `bid` of `nb` (a burst-server workgroup runs its share as block 0 of 1).
__device__ __forceinline__ Sched sched(uint64_t n_iters, bool contig, uint32_t bid, uint32_t nb)
{
	Sched s;
	if (contig) {
		const uint64_t per = (n_iters + nb - 1) / nb;
		s.it = (uint64_t)bid * per;
		s.end = s.it + per < n_iters ? s.it + per : n_iters;
		s.step = 1;
	} else {
		s.it = bid;
		s.end = n_iters;
		s.step = nb;
	}
	return s;
}

__device__ __forceinline__ Sched sched(uint64_t n_iters, bool contig)
{
	return sched(n_iters, contig, blockIdx.x, gridDim.x);
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
		const CGCK_GLOBAL uint32_t *d = (const CGCK_GLOBAL uint32_t *)p.desc + 3 * kk;
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

// The same over descriptors staged in the workgroup's LDS (the burst server's
// slice path): p.desc is a generic pointer into LDS, read as ds_read.
typedef __attribute__((address_space(3))) const uint32_t lds_u32;
typedef __attribute__((address_space(3))) const u32x4_t lds_v4;
typedef __attribute__((address_space(3))) const uint8_t lds_u8;

// Packet bytes from global memory, or (LDSP) from LDS through a generic
// pointer into it (the burst server's small request block, copied into LDS)
template <bool NT, bool LDSP>
__device__ __forceinline__ uint4 ldq(const uint4 *p)
{
	if constexpr (LDSP) {
		const u32x4_t v = *(lds_v4 *)p;
		return make_uint4(v[0], v[1], v[2], v[3]);
	} else {
		return ld<NT>(p);
	}
}

template <bool NT, bool LDSP>
__device__ __forceinline__ uint4 ldcq(const uint4 *c0, int i, int nch, const void *zero)
{
	return ldq<NT, LDSP>(nch > 0 ? c0 + min(i, nch - 1) : reinterpret_cast<const uint4 *>(zero));
}

template <bool LDSP>
__device__ __forceinline__ uint32_t ld8q(uint64_t a)
{
	return LDSP ? (uint32_t) * (lds_u8 *)(const uint8_t *)a : (uint32_t)*gbl_at<const uint8_t>(a);
}
__device__ __forceinline__ Pkt get_pkt_lds(const KParams &p, uint64_t k)
{
	Pkt r;
	r.ok = k < p.n;
	const uint32_t kk = r.ok ? (uint32_t)k : 0u;
	lds_u32 *d = (lds_u32 *)(const uint32_t *)p.desc + 3 * kk;
	const uint32_t lo = d[0], hi = d[1], w2 = d[2];
	r.a0 = reinterpret_cast<uint64_t>(p.base) + (((uint64_t)hi << 32) | lo) + (w2 & 0xffffu);
	r.len = r.ok ? w2 >> 16 : 0u;
	return r;
}

// Is descriptor {lo, hi, w2} (frame_off, l3_off | ip_len << 16) inside a
// range of `limit` bytes: frame_off + l3_off + ip_len <= limit, no wrap.
__device__ __forceinline__ bool desc_inside(uint32_t lo, uint32_t hi, uint32_t w2, uint64_t limit)
{
	const uint64_t fo = ((uint64_t)hi << 32) | lo;
	return fo <= limit && (w2 & 0xffffu) + (w2 >> 16) <= limit - fo;
}

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

// --------------------------------------------------------------------------
// Lane-group partial sums (cgck_group.hip, cgck_stream.hip)
// --------------------------------------------------------------------------

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
			const uint32_t mf = cmask16(co, q + 10, q + 12);
			const uint32_t mg = fo >= 0 ? cmask16(co, q + hl + fo, q + hl + fo + 2) : 0u;
			const uint32_t f = msum16(w, mf, 0);
			const uint32_t g = msum16(w, mg, 0);
			pt.fld += f | (g << 16);
			zero16(w, mf | mg);
		}
		pt.ip = msum16(w, cmask16(co, q, q + hl), pt.ip);
		pt.ps = msum16(w, cmask16(co, q + 12, q + 20), pt.ps);
	}
	if (co >= q && co + 16 <= q + len)
		pt.tot = sum4(w, pt.tot);
	else
		pt.tot = msum16(w, cmask16(co, q, q + len), pt.tot);
}

} // namespace cgck
