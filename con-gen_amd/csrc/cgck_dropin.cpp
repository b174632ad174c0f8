// cgck_dropin.cpp — the drop-in symbols of subr.h:370-374 (in_cksum,
// udp_cksum, toeplitz_hash, rss_hash4) and the two per-thread windows that
// let the stack's own call sites batch without being edited:
//
//  * the RX window (cgck_rx_begin .. cgck_rx_end): at the transport's receive
//    burst one launch computes every frame's header and L4 checksum with the
//    checksum fields read as zero; the stack's verifiers (ip_input.c:45-58,
//    tcp_input.c:75-85, udp_usrreq.c:86-94, ip_icmp.c:187-193,
//    gbtcp/inet.c:142-153 and 319-330) then call in_cksum / udp_cksum on the
//    same header or segment, after zeroing the field themselves, and get the
//    precomputed value back.  Their count / drop policy (t_*_do_incksum
//    0/1/2) runs unchanged;
//  * the TX window (cgck_tx_begin .. cgck_tx_flush): the finalisers'
//    (ip_output.c:61-64, tcp_output.c:416-418, tcp_subr.c:122,
//    gbtcp/tcp.c:370-379) calls on registered ring memory are queued and
//    filled in one launch before the NIC kick.
//
// A call that neither window answers runs the kernel synchronously on the
// thread's own context.  No value is ever computed on the host.
#include <hip/hip_runtime.h>

#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <vector>

#include "cgck_host.h"

using namespace cgck;

namespace {

// --------------------------------------------------------------------------
// Error handler (cgck_set_error_handler)
// --------------------------------------------------------------------------

std::atomic<cgck_error_fn> g_err_fn{nullptr};
std::atomic<void *> g_err_arg{nullptr};

// Open-addressing map from a non-zero key (a pointer, or a pointer times two
// plus a kind bit) to a u32; sized to twice the entries.
struct PtrMap {
	std::vector<uintptr_t> key;
	std::vector<uint32_t> val;
	size_t used = 0;

	static size_t hash(uintptr_t k)
	{
		k ^= k >> 31;
		k *= 0xbf58476d1ce4e5b9ull;
		return (size_t)(k ^ (k >> 29));
	}
	void reset(size_t n)
	{
		size_t cap = 16;
		while (cap < 2 * n)
			cap <<= 1;
		key.assign(cap, 0);
		val.resize(cap);
		used = 0;
	}
	void put(uintptr_t k, uint32_t v)
	{
		if (2 * (used + 1) > key.size()) {
			std::vector<uintptr_t> ok;
			std::vector<uint32_t> ov;
			ok.swap(key);
			ov.swap(val);
			reset(used + 1 < 8 ? 8 : 2 * (used + 1));
			for (size_t i = 0; i < ok.size(); i++)
				if (ok[i])
					put(ok[i], ov[i]);
		}
		const size_t m = key.size() - 1;
		for (size_t i = hash(k) & m;; i = (i + 1) & m)
			if (key[i] == 0 || key[i] == k) {
				used += key[i] == 0;
				key[i] = k;
				val[i] = v;
				return;
			}
	}
	bool get(uintptr_t k, uint32_t *v) const
	{
		if (key.empty())
			return false;
		const size_t m = key.size() - 1;
		for (size_t i = hash(k) & m;; i = (i + 1) & m) {
			if (key[i] == k) {
				*v = val[i];
				return true;
			}
			if (key[i] == 0)
				return false;
		}
	}
};

struct TxEntry {
	uint8_t *ip;   // IPv4 header in registered (ring) memory
	uint32_t span; // bytes from ip the checksum covers
	uint16_t hl;
	int16_t fo; // -1: IP header entry (field ip+10); else L4 field offset after the header
};

// One receive burst: its descriptors and the kernel's values and meta words
// (kFlagRx), and, when it was left posted on the burst server, the request.
struct RxBurst {
	const uint8_t *base = nullptr;
	uint64_t n = 0;
	std::vector<cgck_desc_t> d;
	std::vector<uint32_t> o, m;
	BurstPending pend{};
};

// One TX flush: the queued fields, the descriptors of the in-place batch (or
// the staged copies' values), and the posted request (cgck_tx_post).
struct TxFill {
	std::vector<TxEntry> q;
	std::vector<cgck_desc_t> d;
	std::vector<uint32_t> o, idx; // idx: the value (descriptor) of each queued entry
	BurstPending pend{};
	bool stored = false; // the kernel wrote the fields in place (CGCK_STORE): nothing left to write
	bool fast = false;   // posted in the fast form: o[k] is descriptor k's values, hs its spans
	bool icmp = false;   // holds ICMP messages (their L4 value without the pseudo-header)
	int n = 0;           // the fields it stands for (q is empty in the fast form)
	std::vector<uint32_t> hs;
	uint8_t *lo = nullptr;
};

struct ThreadState {
	cgck_ctx *ctx = nullptr;
	// TX window
	bool tx_open = false;
	bool tx_icmp = false; // an ICMP message was queued (icmp_send, ip_icmp.c:68-80)
	std::vector<TxEntry> txq;
	const uint8_t *tx_max = nullptr; // highest header address queued so far
	bool tx_map = false;             // txidx built (the first call below tx_max)
	PtrMap txidx; // (ip << 1 | is_l4) -> txq index
	TxFill txs;       // cgck_tx_flush's batch
	TxFill txp[2];    // posted fills (cgck_tx_post), oldest at txp_head
	unsigned txp_head = 0, txp_count = 0;
	// The window in its fast form, while every call is at or above the
	// highest header so far and inside one registered range (txd_ok): no
	// txq entries, only one descriptor per packet, its header and segment
	// entries merged, so cgck_tx_post sends them as they are.  txd_h /
	// txd_s: the current packet's header and segment spans (0: not queued),
	// txd_hs the closed packets' (h << 16 | s), from which txd_spill builds
	// txq when the window leaves the fast form; txd_noip: packets whose
	// header was not queued; txd_calls: the entries the window stands for.
	std::vector<cgck_desc_t> txd_fast;
	std::vector<uint32_t> txd_hs;
	bool txd_ok = false;
	const uint8_t *txd_lo = nullptr, *txd_hi = nullptr;
	uint32_t txd_h = 0, txd_s = 0, txd_noip = 0, txd_max = 0, txd_calls = 0;
	size_t txd_bytes = 0; // 16-byte-rounded packet bytes of the closed descriptors
	// RX window: frame i's header at rx_base + rxd[i].frame_off +
	// rxd[i].l3_off; rxo[i] its values (lo16 header checksum, hi16 L4
	// checksum, ICMP without the pseudo-header) and rxm[i] which calls they
	// answer (kFlagRx's meta word: kRxOkIp | kRxOkL4 | kRxIcmp, ip_hl * 4 in
	// bits 8-15, ntohs(ip_len) - ip_hl * 4 in bits 16-31, zero for a frame the
	// stack drops before any checksum), both written by the kernel; they point
	// into the burst the window answers from
	bool rx_open = false;
	bool rx_posted = false; // the window is over the oldest posted burst
	const uint8_t *rx_base = nullptr;
	size_t rx_n = 0;
	size_t rx_cur = 0;    // the frame the last answered call matched
	bool rx_map = false;  // rxidx built (on the first call off the cursor)
	PtrMap rxidx; // ip -> frame << 1; ip + hl (ICMP message) -> frame << 1 | 1
	const cgck_desc_t *rxd = nullptr;
	const uint32_t *rxo = nullptr, *rxm = nullptr;
	// the burst's frames as sorted [start, end) byte ranges, built on the
	// first TX-window call of the window (rx_owns)
	bool rx_iv_built = false;
	std::vector<std::pair<uintptr_t, uintptr_t>> rx_iv;
	RxBurst rxs;      // cgck_rx_begin's burst
	RxBurst rxp[2];   // posted bursts (cgck_rx_post), oldest at rxp_head
	unsigned rxp_head = 0, rxp_count = 0;
	uint64_t rx_served0 = 0; // stats[0] at rx_begin
	uint64_t stats[4] = {0, 0, 0, 0};
	// the registered range of the last TX-window hit, valid while g_reg_gen
	// holds reg_gen (the window's per-call check without a call out)
	RegRange reg_last{nullptr, nullptr, nullptr};
	uint64_t reg_gen = 0;
};

// The drop-ins read this on every call, so it is a plain pointer in the
// initial-exec TLS model (one fs-relative load; a thread_local object with a
// constructor costs a TLS wrapper call and an init guard per access).  The
// state itself is allocated on the thread's first use and freed by
// cgck_thread_release, which keeps only the counters.
__attribute__((tls_model("initial-exec"))) thread_local ThreadState *t_st = nullptr;
// the window counters of a released state (cgck_thread_release frees the state)
__attribute__((tls_model("initial-exec"))) thread_local uint64_t t_stats_kept[4] = {0, 0, 0, 0};

ThreadState &tstate()
{
	if (__builtin_expect(!t_st, 0)) {
		t_st = new ThreadState;
		memcpy(t_st->stats, t_stats_kept, sizeof(t_stats_kept));
	}
	return *t_st;
}

uint32_t sync_region(const void *src, uint32_t span, uint32_t ip_len, uint32_t flags)
{
	cgck_ctx *c = thread_ctx();
	if (!c)
		die("no gfx950 context for the drop-in checksum");
	uint32_t out = 0;
	if (one_region(c, src, span, ip_len, flags, &out) != 0)
		die("drop-in checksum kernel");
	return out;
}

// The window frame a pointer names: (frame << 1) for an IPv4 header,
// (frame << 1 | 1) for the ICMP message after it.  The stack walks a burst in
// slot order and asks for each frame's header and then its segment, so the
// frame of the previous answer or the next answerable one almost always
// matches; a map of every frame is built only on the first call that matches
// neither.
inline const uint8_t *rx_ip(const ThreadState &t, size_t i)
{
	return t.rx_base + t.rxd[i].frame_off + t.rxd[i].l3_off;
}

__attribute__((noinline)) bool rx_find_slow(ThreadState &t, const uint8_t *p, uint32_t *v)
{
	const size_t n = t.rx_n;
	const uint32_t *m = t.rxm;
	// the cursor frame, then the next answerable ones (frames the stack
	// dropped unverified have no calls: up to 8 are stepped over)
	for (size_t i = t.rx_cur, seen = 0, lim = t.rx_cur + 10; i < n && i < lim && seen < 2; i++) {
		if (!m[i])
			continue;
		seen++;
		const uint8_t *ip = rx_ip(t, i);
		if (ip == p) {
			*v = (uint32_t)(i << 1);
			t.rx_cur = i;
			return true;
		}
		if ((m[i] & kRxIcmp) && ip + (m[i] >> 8 & 0xff) == p) {
			*v = (uint32_t)(i << 1 | 1);
			t.rx_cur = i;
			return true;
		}
	}
	if (!t.rx_map) {
		t.rxidx.reset(2 * n);
		for (size_t i = 0; i < n; i++) {
			if (!m[i])
				continue;
			const uint8_t *ip = rx_ip(t, i);
			t.rxidx.put((uintptr_t)ip, (uint32_t)(i << 1));
			if ((m[i] & (kRxIcmp | kRxOkL4)) == (kRxIcmp | kRxOkL4))
				t.rxidx.put((uintptr_t)(ip + (m[i] >> 8 & 0xff)), (uint32_t)(i << 1 | 1));
		}
		t.rx_map = true;
	}
	if (!t.rxidx.get((uintptr_t)p, v))
		return false;
	t.rx_cur = *v >> 1;
	return true;
}

// The header of the cursor frame or of the next one (the stack's next call
// is almost always one of the two) without leaving the caller; everything
// else (ICMP messages, skipped frames, the map) in rx_find_slow.
inline bool rx_find(ThreadState &t, const uint8_t *p, uint32_t *v)
{
	const size_t i = t.rx_cur;
	if (__builtin_expect(i + 1 < t.rx_n, 1)) {
		if (t.rxm[i] && rx_ip(t, i) == p) {
			*v = (uint32_t)(i << 1);
			return true;
		}
		if (t.rxm[i + 1] && rx_ip(t, i + 1) == p) {
			*v = (uint32_t)((i + 1) << 1);
			t.rx_cur = i + 1;
			return true;
		}
	}
	return rx_find_slow(t, p, v);
}

// The L4 checksum field after the IPv4 header, by protocol, as the
// finalisers store it: TCP +16 (tcp_output.c:417), UDP +6 (udp_usrreq.c:
// 189), ICMP +2 (icmp_send, ip_icmp.c:76-77).
inline int l4_fo(const uint8_t *ip) { return ip[9] == 6 ? 16 : ip[9] == 17 ? 6 : 2; }

// Does p lie inside one of the open RX window's frames?  Both windows are
// open across con-gen's whole loop iteration, so a
// call the RX window does not answer may still be the stack verifying a
// received frame (a UDP datagram whose uh_ulen is below ip_len, an ICMP
// message too short to check); it needs its value now, so it must not be
// queued by the TX window even though the frame lies in the registered
// pool.  The frames' ranges are sorted once per window, on the first call
// that asks (a burst that draws no reply never pays for it).
__attribute__((noinline)) bool rx_owns(ThreadState &t, const uint8_t *p)
{
	if (!t.rx_iv_built) {
		t.rx_iv.resize(t.rx_n);
		bool sorted = true;
		for (size_t i = 0; i < t.rx_n; i++) {
			const uintptr_t a = (uintptr_t)(t.rx_base + t.rxd[i].frame_off);
			t.rx_iv[i] = {a, a + t.rxd[i].l3_off + t.rxd[i].ip_len};
			sorted = sorted && (i == 0 || t.rx_iv[i - 1].first <= a);
		}
		if (!sorted)
			std::sort(t.rx_iv.begin(), t.rx_iv.end());
		// a running maximum of the ends, so one probe answers for overlaps
		for (size_t i = 1; i < t.rx_n; i++)
			t.rx_iv[i].second = std::max(t.rx_iv[i].second, t.rx_iv[i - 1].second);
		t.rx_iv_built = true;
	}
	const uintptr_t a = (uintptr_t)p;
	auto it = std::upper_bound(t.rx_iv.begin(), t.rx_iv.end(), std::make_pair(a, UINTPTR_MAX));
	return it != t.rx_iv.begin() && (it - 1)->second > a;
}

// Is [p, p + bytes) registered (the TX window queues only ring memory)?  The
// range of the last hit first, then reg_find.  The generation is read before
// the lookup, so a change racing it leaves the cache stale-marked.
inline bool tx_registered(ThreadState &t, const uint8_t *p, size_t bytes)
{
	const uint64_t g = g_reg_gen.load(std::memory_order_acquire);
	if (__builtin_expect(t.reg_gen == g && p >= t.reg_last.lo && p < t.reg_last.hi &&
			     bytes <= (size_t)(t.reg_last.hi - p), 1))
		return true;
	RegRange r;
	if (!reg_find(p, bytes, &r))
		return false;
	t.reg_last = r;
	t.reg_gen = g;
	return true;
}

// The current packet's descriptor closed: its spans, its length and whether
// its header was queued enter the window's summary.
__attribute__((always_inline)) inline void txd_close(ThreadState &t)
{
	if (t.txd_fast.size() == t.txd_hs.size())
		return; // none open
	const uint32_t len = t.txd_fast.back().ip_len;
	t.txd_hs.push_back(t.txd_h << 16 | t.txd_s);
	t.txd_noip += t.txd_h == 0;
	t.txd_max = len > t.txd_max ? len : t.txd_max;
	t.txd_bytes += (len + 15) & ~15u;
}

// Leave the fast form: txq rebuilt from the descriptors, per packet its
// segment entry then its header entry, as the finalisers queue them
// (tcp_output.c:416-418 before ip_output.c:61-64).  A segment entry's header
// length and protocol are read from the packet again, as its call read them.
__attribute__((noinline)) void txd_spill(ThreadState &t)
{
	const size_t n = t.txd_fast.size();
	t.txq.clear();
	for (size_t k = 0; k < n; k++) {
		const uint32_t hs = k < t.txd_hs.size() ? t.txd_hs[k] : (t.txd_h << 16 | t.txd_s);
		uint8_t *ip = const_cast<uint8_t *>(t.txd_lo) + t.txd_fast[k].frame_off;
		const uint32_t h = hs >> 16, sp = hs & 0xffff;
		if (sp)
			t.txq.push_back({ip, sp, (uint16_t)((ip[0] & 15) * 4), (int16_t)l4_fo(ip)});
		if (h)
			t.txq.push_back({ip, h, (uint16_t)h, -1});
	}
	t.txd_ok = false;
	t.txd_fast.clear();
	t.txd_hs.clear();
}

// Queue one field; a header or segment queued again replaces its entry (the
// later call wins).  The transport hands out ring slots in address order, so
// while every call is at or above the highest header queued so far a
// duplicate can only be the current packet's (the fast form keeps only the
// descriptors; the general form scans the last entries); the first call
// below it (ring wrap, a slot handed out again) switches to a map of every
// entry.  tx_queue: the fast form's two common calls (the next packet in
// the range, the current packet's other entry) inline in the drop-ins; the
// window's first call and everything else here.
__attribute__((noinline)) void tx_queue_slow(ThreadState &t, uint8_t *ip, uint32_t span, uint16_t hl, int16_t fo)
{
	const TxEntry e = {ip, span, hl, fo};
	if (!t.tx_map) {
		if (ip > t.tx_max) {
			t.tx_max = ip;
			if (t.txd_ok) {
				if (t.txd_fast.empty()) { // the range of the window's first call
					t.txd_lo = t.reg_last.lo;
					t.txd_hi = t.reg_last.hi;
				}
				if (ip >= t.txd_lo && ip + span <= t.txd_hi) {
					txd_close(t);
					t.txd_fast.push_back({(uint64_t)(ip - t.txd_lo), 0, (uint16_t)span});
					t.txd_h = fo < 0 ? span : 0;
					t.txd_s = fo < 0 ? 0 : span;
					t.txd_calls++;
					return;
				}
				txd_spill(t); // a second range: the post builds the batch
			}
			t.txq.push_back(e);
			return;
		}
		if (ip == t.tx_max) {
			if (t.txd_ok) { // the current packet's other entry, or a later call for the same one
				uint32_t &sp = fo < 0 ? t.txd_h : t.txd_s;
				t.txd_calls += sp == 0;
				sp = span;
				t.txd_fast.back().ip_len = (uint16_t)(t.txd_h > t.txd_s ? t.txd_h : t.txd_s);
				return;
			}
			for (size_t i = t.txq.size(); i-- > 0 && t.txq[i].ip == ip;)
				if ((t.txq[i].fo < 0) == (fo < 0)) {
					t.txq[i] = e;
					return;
				}
			t.txq.push_back(e);
			return;
		}
		if (t.txd_ok) // out of address order: the map, and the post builds the batch
			txd_spill(t);
		t.txidx.reset(2 * t.txq.size() + 64);
		for (size_t i = 0; i < t.txq.size(); i++)
			t.txidx.put(((uintptr_t)t.txq[i].ip << 1) | (t.txq[i].fo >= 0 ? 1u : 0u), (uint32_t)i);
		t.tx_map = true;
	}
	const uintptr_t k = ((uintptr_t)ip << 1) | (fo >= 0 ? 1u : 0u);
	uint32_t i;
	if (t.txidx.get(k, &i)) {
		t.txq[i] = e;
		return;
	}
	t.txidx.put(k, (uint32_t)t.txq.size());
	t.txq.push_back(e);
}

__attribute__((always_inline)) inline void tx_queue(ThreadState &t, uint8_t *ip, uint32_t span, uint16_t hl,
						     int16_t fo)
{
	if (__builtin_expect(t.txd_ok, 1)) {
		// (a non-empty fast form: txd_lo <= tx_max, so ip > tx_max is in the range from below)
		if (ip > t.tx_max && !t.txd_fast.empty() && ip + span <= t.txd_hi) {
			t.tx_max = ip;
			txd_close(t);
			t.txd_fast.push_back({(uint64_t)(ip - t.txd_lo), 0, (uint16_t)span});
			t.txd_h = fo < 0 ? span : 0;
			t.txd_s = fo < 0 ? 0 : span;
			t.txd_calls++;
			return;
		}
		if (ip == t.tx_max) {
			uint32_t &sp = fo < 0 ? t.txd_h : t.txd_s;
			t.txd_calls += sp == 0;
			sp = span;
			t.txd_fast.back().ip_len = (uint16_t)(t.txd_h > t.txd_s ? t.txd_h : t.txd_s);
			return;
		}
	}
	tx_queue_slow(t, ip, span, hl, fo);
}

} // namespace

// --------------------------------------------------------------------------
// Per-thread context and failure reporting
// --------------------------------------------------------------------------

cgck_ctx *cgck::thread_ctx()
{
	ThreadState &t = tstate();
	if (!t.ctx) {
		const char *e = getenv("CGCK_DEVICE");
		const int dev = e ? atoi(e) : 0;
		cgck_ctx *c = nullptr;
		if (cgck_ctx_create(dev, &c) != 0)
			return nullptr;
		t.ctx = c;
	}
	return t.ctx;
}

cgck_ctx *cgck::thread_ctx_if_any() { return t_st ? t_st->ctx : nullptr; }

[[noreturn]] void cgck::die(const char *what)
{
	const cgck_error_fn fn = g_err_fn.load(std::memory_order_acquire);
	void *arg = g_err_arg.load(std::memory_order_acquire);
	if (fn)
		fn(what, err_text(), arg);
	fprintf(stderr, "libcgck: %s: %s\n", what, err_text());
	abort();
}

extern "C" void cgck_set_error_handler(cgck_error_fn fn, void *arg)
{
	g_err_arg.store(arg, std::memory_order_release);
	g_err_fn.store(fn, std::memory_order_release);
}

extern "C" cgck_ctx_t *cgck_thread_ctx(void) { return thread_ctx(); }

extern "C" int cgck_thread_release(void)
{
	ThreadState *t = t_st;
	if (!t)
		return 0;
	if (t->ctx)
		cgck_ctx_destroy(t->ctx);
	// Only the counters outlive the release (cgck_window_stats, in plain
	// TLS): the state with its window queues, maps and burst-sized buffers is
	// freed, so a pool that retires threads keeps nothing per thread.
	memcpy(t_stats_kept, t->stats, sizeof(t_stats_kept));
	delete t;
	t_st = nullptr;
	return 0;
}

extern "C" int cgck_window_stats(uint64_t stats[4])
{
	if (!stats)
		return set_err(-EINVAL, "cgck_window_stats: NULL");
	memcpy(stats, t_st ? t_st->stats : t_stats_kept, sizeof(t_stats_kept));
	return 0;
}

// --------------------------------------------------------------------------
// Drop-in symbols (subr.h:373-374; bodies subr.c:186-195, 212-223)
// --------------------------------------------------------------------------

extern "C" uint16_t in_cksum(void *data, int len)
{
	if (len < 0) {
		// The reference's cksum_raw never terminates sensibly on a negative
		// size (subr.c:164 compares it as size_t); refuse loudly instead.
		set_err(-EINVAL, "in_cksum: negative length %d", len);
		die("in_cksum");
	}
	ThreadState &t = tstate();
	const uint8_t *b = (const uint8_t *)data;
	bool rx_miss = false; // counted in stats[1] only when the call is computed here
	bool rx_frame = false; // the call is about a received frame: never queued
	if (t.rx_open) {
		// ip_cksum(ip) at ip_input.c:51 / inet.c:322, or the ICMP message at
		// ip_icmp.c:189, after the caller zeroed the field
		uint32_t v;
		if (rx_find(t, b, &v)) {
			const uint32_t m = t.rxm[v >> 1];
			if (!(v & 1) && (m & kRxOkIp) && (uint32_t)len == (m >> 8 & 0xff)) {
				t.stats[0]++;
				return (uint16_t)t.rxo[v >> 1];
			}
			if ((v & 1) && (m & kRxOkL4) && (uint32_t)len == m >> 16) {
				t.stats[0]++;
				return (uint16_t)(t.rxo[v >> 1] >> 16);
			}
			rx_frame = true;
		}
		rx_miss = true;
	}
	if (t.tx_open && !rx_frame && !(rx_miss && rx_owns(t, b))) {
		if (len >= 20 && (b[0] >> 4) == 4 && len == (b[0] & 15) * 4) {
			// ip_cksum(ip) in ip_output (ip_output.c:62)
			if (tx_registered(t, b, (size_t)len)) {
				tx_queue(t, (uint8_t *)data, (uint32_t)len, (uint16_t)len, -1);
				t.stats[2]++;
				return 0;
			}
			t.stats[3]++;
		} else if (len >= 8 && len <= 0xffff - 20) {
			// icmp_send's in_cksum(icp, ip_len - 20) (ip_icmp.c:77): the
			// message right after a 20-byte IPv4 header of protocol 1, its
			// field at +2 just zeroed; queued as the packet's L4 entry.  The
			// header bytes are read only when they are registered or on
			// the message's own page.
			const uint8_t *ip = b - 20;
			if (tx_registered(t, ip, 20 + (size_t)len)) {
				if (ip[0] == 0x45 && ip[9] == 1) {
					tx_queue(t, const_cast<uint8_t *>(ip), 20 + (uint32_t)len, 20, 2);
					t.tx_icmp = true;
					t.stats[2]++;
					return 0;
				}
			} else if (((uintptr_t)b & 4095) >= 20 && ip[0] == 0x45 && ip[9] == 1) {
				t.stats[3]++;
			}
		}
	}
	t.stats[1] += rx_miss;
	return (uint16_t)sync_region(data, (uint32_t)len, (uint32_t)len, CGCK_RAW);
}

extern "C" uint16_t udp_cksum(struct ip *ipp, int len)
{
	const uint8_t *ip = (const uint8_t *)ipp;
	if (len < 0) {
		set_err(-EINVAL, "udp_cksum: negative length %d", len);
		die("udp_cksum");
	}
	ThreadState &t = tstate();
	const uint32_t hl = (ip[0] & 15) * 4;
	const uint32_t ip_len = hl + (uint32_t)len;
	bool rx_miss = false; // counted in stats[1] only when the call is computed here
	bool rx_frame = false; // the call is about a received frame: never queued
	if (t.rx_open) {
		// tcp_cksum(ip, ip->ip_len) at tcp_input.c:78 / inet.c:145, or
		// udp_cksum(ip, len) at udp_usrreq.c:89
		uint32_t v;
		if (rx_find(t, ip, &v)) {
			const uint32_t m = t.rxm[v >> 1];
			if (!(v & 1) && (m & (kRxOkL4 | kRxIcmp)) == kRxOkL4 && (uint32_t)len == m >> 16 &&
			    hl == (m >> 8 & 0xff)) {
				t.stats[0]++;
				return (uint16_t)(t.rxo[v >> 1] >> 16);
			}
			rx_frame = true;
		}
		rx_miss = true;
	}
	if (t.tx_open && !rx_frame && hl >= 20 && ip_len <= 0xffff && (ip[9] == 6 || ip[9] == 17) &&
	    !(rx_miss && rx_owns(t, ip))) {
		const int fo = ip[9] == 6 ? 16 : 6;
		if ((uint32_t)len >= (uint32_t)fo + 2) {
			if (tx_registered(t, ip, ip_len)) {
				tx_queue(t, (uint8_t *)ip, ip_len, (uint16_t)hl, (int16_t)fo);
				t.stats[2]++;
				return 0;
			}
			t.stats[3]++;
		}
	}
	// The pseudo-header reads ip+9 and ip+12..19 whatever ip_hl says
	// (subr.c:205-207), so at least 20 bytes are staged.
	const uint32_t span = ip_len < 20 ? 20 : ip_len;
	t.stats[1] += rx_miss;
	return (uint16_t)(sync_region(ip, span, ip_len, CGCK_L4 | kFlagNoLenCheck) >> 16);
}

// --------------------------------------------------------------------------
// RX window
// --------------------------------------------------------------------------

namespace {

constexpr uint32_t kRxFlags = CGCK_IP | CGCK_L4 | CGCK_ZERO_FIELDS | kFlagL4Auto | kFlagRx;

// Fill a burst's descriptor copy and output arrays for n frames.
void rx_fill(RxBurst &r, const void *base, const cgck_desc_t *desc, uint64_t n)
{
	r.base = (const uint8_t *)base;
	r.n = n;
	r.d.assign(desc, desc + n);
	r.o.resize(n ? n : 1);
	r.m.resize(n ? n : 1);
}

// Open the window over a computed burst; returns the frames it answers for.
int rx_open_on(ThreadState &t, const RxBurst &r, bool posted)
{
	uint64_t m = 0;
	for (uint64_t i = 0; i < r.n; i++)
		m += r.m[i] != 0;
	t.rxd = r.d.data();
	t.rxo = r.o.data();
	t.rxm = r.m.data();
	t.rx_base = r.base;
	t.rx_n = r.n;
	t.rx_cur = 0;
	t.rx_map = false;
	t.rx_iv_built = false;
	t.rx_open = true;
	t.rx_posted = posted;
	t.rx_served0 = t.stats[0];
	return (int)m;
}

int rx_check(ThreadState &t, const void *base, const cgck_desc_t *desc, uint64_t n, const char *who)
{
	(void)t;
	if (n && (!base || !desc))
		return set_err(-EINVAL, "%s: NULL base or descriptors", who);
	if (n > 0xffffffffull / 2)
		return set_err(-EINVAL, "%s: burst of %llu frames", who, (unsigned long long)n);
	return 0;
}

} // namespace

extern "C" int cgck_rx_begin(void *base, size_t bytes, const cgck_desc_t *desc, uint64_t n)
{
	ThreadState &t = tstate();
	if (t.rx_open)
		return set_err(-EBUSY, "cgck_rx_begin: an RX window is already open on this thread");
	int rc = rx_check(t, base, desc, n, "cgck_rx_begin");
	if (rc)
		return rc;
	cgck_ctx *c = thread_ctx();
	if (!c)
		return -ENODEV; // thread_ctx set the message
	// One launch (or one burst-server request) over the whole burst: the
	// kernel sums each frame's header and L4 checksum with the fields read as
	// zero (ICMP without the pseudo-header) and itself decides, from the
	// frame's header, which calls the stack can make on it (kFlagRx: the
	// drop rules of ip_input.c:28-44, 76, tcp_input.c:67, udp_usrreq.c:65,
	// ip_icmp.c:177, gbtcp/inet.c:282-314), so no header is parsed here.
	// desc_host checks every descriptor against [base, base + bytes).
	rx_fill(t.rxs, base, desc, n);
	if (n && (rc = desc_host(c, base, bytes, t.rxs.d.data(), n, kRxFlags, t.rxs.o.data(), nullptr,
				 t.rxs.m.data()))) {
		char msg[256];
		snprintf(msg, sizeof(msg), "%s", err_text());
		return set_err(rc, "cgck_rx_begin: %s", msg);
	}
	return rx_open_on(t, t.rxs, false);
}

// Pipelined form: post burst k and return; the window over it opens at a
// later cgck_rx_begin_posted, while the stack has worked on burst k - 1.
extern "C" int cgck_rx_post(void *base, size_t bytes, const cgck_desc_t *desc, uint64_t n)
{
	ThreadState &t = tstate();
	if (t.rxp_count == 2)
		return set_err(-EBUSY, "cgck_rx_post: two bursts already posted and not yet opened");
	int rc = rx_check(t, base, desc, n, "cgck_rx_post");
	if (rc)
		return rc;
	cgck_ctx *c = thread_ctx();
	if (!c)
		return -ENODEV;
	RxBurst &r = t.rxp[(t.rxp_head + t.rxp_count) & 1];
	rx_fill(r, base, desc, n);
	r.pend.seq = 0;
	r.pend.rc = 0;
	if (n && (rc = desc_host_post(c, base, bytes, r.d.data(), n, kRxFlags, r.o.data(), nullptr, r.m.data(),
				      &r.pend)) < 0) {
		char msg[256];
		snprintf(msg, sizeof(msg), "%s", err_text());
		return set_err(rc, "cgck_rx_post: %s", msg);
	}
	t.rxp_count++;
	return (int)n;
}

extern "C" int cgck_rx_begin_posted(void)
{
	ThreadState &t = tstate();
	if (t.rx_open)
		return set_err(-EBUSY, "cgck_rx_begin_posted: an RX window is already open on this thread");
	if (t.rxp_count == 0)
		return set_err(-ENOENT, "cgck_rx_begin_posted: no burst posted");
	RxBurst &r = t.rxp[t.rxp_head];
	int rc = r.pend.seq ? burst_collect(t.ctx, &r.pend) : r.pend.rc;
	if (rc) {
		t.rxp_head ^= 1;
		t.rxp_count--;
		char msg[256];
		snprintf(msg, sizeof(msg), "%s", err_text());
		return set_err(rc, "cgck_rx_begin_posted: %s", msg);
	}
	return rx_open_on(t, r, true);
}

// The drain rule's two questions (include/cgck.h): is a burst still posted,
// and would opening the oldest one wait for the GPU?
extern "C" int cgck_rx_pending(void)
{
	const ThreadState *t = t_st;
	return t ? (int)t->rxp_count : 0;
}

extern "C" int cgck_rx_ready(void)
{
	const ThreadState *t = t_st;
	if (!t || t->rxp_count == 0)
		return set_err(-ENOENT, "cgck_rx_ready: no burst posted");
	const RxBurst &r = t->rxp[t->rxp_head];
	return r.pend.seq ? burst_ready(t->ctx, &r.pend) : 1;
}

extern "C" int cgck_rx_end(void)
{
	ThreadState &t = tstate();
	if (!t.rx_open)
		return set_err(-EINVAL, "cgck_rx_end: no open RX window on this thread");
	t.rx_open = false;
	t.rx_n = 0;
	t.rx_map = false;
	if (t.rx_posted) {
		t.rx_posted = false;
		t.rxp_head ^= 1;
		t.rxp_count--;
	}
	return (int)(t.stats[0] - t.rx_served0);
}

// --------------------------------------------------------------------------
// TX window
// --------------------------------------------------------------------------

extern "C" int cgck_tx_begin(void)
{
	ThreadState &t = tstate();
	if (t.tx_open)
		return set_err(-EBUSY, "cgck_tx_begin: window already open on this thread");
	t.tx_open = true;
	t.tx_icmp = false;
	t.txq.clear();
	t.tx_max = nullptr;
	t.tx_map = false;
	t.txd_fast.clear();
	t.txd_hs.clear();
	t.txd_ok = true;
	t.txd_h = t.txd_s = t.txd_noip = t.txd_max = t.txd_calls = 0;
	t.txd_bytes = 0;
	return 0;
}

namespace {

// Both kinds in one batch: IP entries ask for the header checksum, L4
// entries for the segment checksum; both read their fields as zero, as the
// reference's callers have just stored them (ip_output.c:61, tcp_subr.c:75 /
// gbtcp/tcp.c:426,436).
constexpr uint32_t kTxFlags = CGCK_IP | CGCK_L4 | CGCK_ZERO_FIELDS;

// A fill with ICMP messages also asks for their values without the
// pseudo-header (kFlagL4Auto: by ip_p, as the RX window does); TCP and UDP
// keep it.  Only then, because the lane-per-packet kernels take no
// kFlagL4Auto and the group kernel is slower on small frames.
inline uint32_t tx_flags(const TxFill &f) { return kTxFlags | (f.icmp ? kFlagL4Auto : 0u); }

// Posted fills return values and the completion writes the fields on the
// host (see cgck_tx_post); the lab build's $CGCK_TX_KSTORE has the kernel
// store them instead (CGCK_STORE), for the A/B.
inline bool tx_kstore()
{
	static const bool k = CGCK_ENV("CGCK_TX_KSTORE") != nullptr;
	return k;
}

// Compute the values of f.q: when every entry lies in one registered range
// (the transport's pool) the batch is described in place, as cgck_desc_host
// of that range — the burst server when one is open on this context and the
// flush fits it (left posted when pend is given: returns 1), else a launch;
// otherwise each region is staged 16-byte aligned in pinned memory and
// launched (computed at once: 0).  f.idx[i] is entry i's value in f.o.
int tx_compute(cgck_ctx *c, TxFill &f, bool post)
{
	const std::vector<TxEntry> &q = f.q;
	const uint64_t n = q.size();
	const uint32_t flags = tx_flags(f);
	HIP_TRY(hipSetDevice(c->device));
	RegRange reg{nullptr, nullptr, nullptr};
	bool inplace = reg_find(q[0].ip, q[0].span, &reg);
	for (uint64_t i = 1; inplace && i < n; i++)
		inplace = q[i].ip >= reg.lo && q[i].ip + q[i].span <= reg.hi;
	int rc;
	// One descriptor per packet: a packet's header entry and its segment
	// entry (queued one after the other by the finalisers, ip_output.c:61-64
	// after tcp_output.c:416-418) share it — it covers the segment, and the
	// kernel returns both the header checksum (over ip_hl * 4 bytes, which
	// the queue checked equals the header call's length) and the segment's
	// L4 checksum from one read of the frame.
	f.idx.resize(n);
	f.stored = false;
	if (inplace) {
		f.d.resize(n);
		uint64_t m = 0;
		bool l4_alone = false; // a packet with its segment queued but not its header
		for (uint64_t i = 0; i < n; i++) {
			if (i > 0 && q[i].ip == q[i - 1].ip && (q[i].fo < 0) != (q[i - 1].fo < 0) && f.idx[i - 1] == m - 1 &&
			    (i < 2 || f.idx[i - 2] != m - 1)) {
				f.idx[i] = (uint32_t)(m - 1);
				if (q[i].span > f.d[m - 1].ip_len)
					f.d[m - 1].ip_len = (uint16_t)q[i].span;
				continue;
			}
			if (q[i].fo >= 0 && !(i + 1 < n && q[i + 1].ip == q[i].ip && q[i + 1].fo < 0))
				l4_alone = true;
			f.idx[i] = (uint32_t)m;
			f.d[m].frame_off = (uint64_t)(q[i].ip - reg.lo);
			f.d[m].l3_off = 0;
			f.d[m].ip_len = (uint16_t)q[i].span;
			m++;
		}
		f.o.resize(m);
		if (post) {
			// Posted: completing the fill writes the fields from the values
			// (tx_write).  Lab ($CGCK_TX_KSTORE): when every packet's header
			// is queued (alone, or with its segment), the kernel stores them
			// (CGCK_STORE: ip+10, and the L4 field of a descriptor that
			// covers the segment; a header-only descriptor covers
			// ip_hl * 4 bytes, so no L4 field fits in it and none is stored).
			f.stored = tx_kstore() && !l4_alone;
			return desc_host_post(c, reg.lo, (size_t)(reg.hi - reg.lo), f.d.data(), m,
					      flags | (f.stored ? CGCK_STORE : 0u), f.stored ? nullptr : f.o.data(), nullptr,
					      nullptr, &f.pend);
		}
		return desc_host(c, reg.lo, (size_t)(reg.hi - reg.lo), f.d.data(), m, flags, f.o.data(), nullptr);
	}
	for (uint64_t i = 0; i < n; i++)
		f.idx[i] = (uint32_t)i;
	size_t bytes = 0; // staged bytes
	for (const TxEntry &e : q)
		bytes += (e.span + 15) & ~(size_t)15;
	const size_t d_off = (bytes + 15) & ~(size_t)15;
	const size_t o_off = (d_off + 12 * n + 15) & ~(size_t)15;
	if ((rc = grow_host((void **)&c->h_stage, &c->h_stage_cap, o_off + 4 * n)))
		return rc;
	uint8_t *h = c->h_stage;
	cgck_desc_t *d = (cgck_desc_t *)(h + d_off);
	uint32_t *o = (uint32_t *)(h + o_off);
	size_t at = 0;
	for (uint64_t i = 0; i < n; i++) {
		memcpy(h + at, q[i].ip, q[i].span);
		d[i].frame_off = at;
		d[i].l3_off = 0;
		d[i].ip_len = (uint16_t)q[i].span;
		at += (q[i].span + 15) & ~(size_t)15;
	}
	KParams p = {h, d, n, 0, 0, 0, flags, o, nullptr, nullptr, 0, nullptr};
	if ((rc = run(c, p, 1500, c->stream)))
		return rc;
	HIP_TRY(hipStreamSynchronize(c->stream));
	f.o.assign(o, o + n);
	return 0;
}

// Write every queued field from the computed values; returns their count.
int tx_write(TxFill &f)
{
	const std::vector<TxEntry> &q = f.q;
	const uint64_t n = q.size();
	for (uint64_t i = 0; i < n; i++) {
		uint16_t v;
		uint8_t *dst;
		const uint32_t r = f.o[f.idx[i]];
		if (q[i].fo < 0) {
			v = (uint16_t)r;
			dst = q[i].ip + 10;
		} else {
			v = (uint16_t)(r >> 16);
			dst = q[i].ip + q[i].hl + q[i].fo;
		}
		memcpy(dst, &v, 2);
	}
	f.q.clear();
	return (int)n;
}

// The fields of a fill posted in the fast form, from descriptor k's values:
// its header's (ip+10) when the header was queued, its segment's when the
// segment was (at ip_hl * 4 + 16 for TCP, + 6 for UDP, read from the packet
// as the call read them).
int tx_write_fast(TxFill &f)
{
	const size_t m = f.d.size();
	for (size_t k = 0; k < m; k++) {
		uint8_t *ip = f.lo + f.d[k].frame_off;
		const uint32_t r = f.o[k], hs = f.hs[k];
		if (hs & 0xffff) {
			const uint16_t v = (uint16_t)(r >> 16);
			memcpy(ip + (ip[0] & 15) * 4 + l4_fo(ip), &v, 2);
		}
		if (hs >> 16) {
			const uint16_t v = (uint16_t)r;
			memcpy(ip + 10, &v, 2);
		}
	}
	return f.n;
}

// Close the window and move its queue into f.
void tx_take(ThreadState &t, TxFill &f)
{
	t.tx_open = false;
	t.tx_map = false;
	f.icmp = t.tx_icmp;
	f.q.swap(t.txq);
	t.txq.clear();
}

} // namespace

extern "C" int cgck_tx_flush(void)
{
	ThreadState &t = tstate();
	if (!t.tx_open)
		return set_err(-EINVAL, "cgck_tx_flush: no open window on this thread");
	txd_close(t);
	if (t.txd_ok && t.txd_noip == 0 && !t.txd_fast.empty()) {
		// the fast form: its descriptors as they are, the fields written from
		// the values (as cgck_tx_post + cgck_tx_complete, waited for at once)
		TxFill &f = t.txs;
		tx_take(t, f);
		cgck_ctx *c = thread_ctx();
		if (!c)
			return -ENODEV;
		f.d.swap(t.txd_fast);
		f.hs.swap(t.txd_hs);
		f.lo = const_cast<uint8_t *>(t.txd_lo);
		f.n = (int)t.txd_calls;
		f.o.resize(f.d.size());
		const DescSummary sum = {t.txd_max, t.txd_bytes};
		int rc = desc_host_post(c, (void *)t.txd_lo, (size_t)(t.txd_hi - t.txd_lo), f.d.data(), f.d.size(),
					tx_flags(f), f.o.data(), nullptr, nullptr, &f.pend, &sum);
		if (rc >= 0)
			rc = f.pend.seq ? burst_collect(c, &f.pend) : f.pend.rc;
		f.q.clear();
		return rc < 0 ? rc : tx_write_fast(f);
	}
	if (t.txd_ok)
		txd_spill(t);
	tx_take(t, t.txs);
	if (t.txs.q.empty())
		return 0;
	cgck_ctx *c = thread_ctx();
	if (!c)
		return -ENODEV;
	int rc = tx_compute(c, t.txs, false);
	if (rc < 0) {
		t.txs.q.clear();
		return rc;
	}
	return tx_write(t.txs);
}

// Pipelined form: post the window's fill and return; cgck_tx_complete
// (before the transport hands these slots to the NIC) waits for it and
// writes the fields.
extern "C" int cgck_tx_post(void)
{
	ThreadState &t = tstate();
	if (!t.tx_open)
		return set_err(-EINVAL, "cgck_tx_post: no open window on this thread");
	if (t.txp_count == 2) {
		// A third fill: the oldest completes first (its fields are written
		// now, before the kick that was to wait for them — final values
		// either way), so no queued field is dropped.
		const int rc = cgck_tx_complete();
		if (rc < 0) {
			t.tx_open = false;
			t.txq.clear();
			char msg[256];
			snprintf(msg, sizeof(msg), "%s", err_text());
			return set_err(rc, "cgck_tx_post: completing the oldest fill: %s", msg);
		}
	}
	TxFill &f = t.txp[(t.txp_head + t.txp_count) & 1];
	txd_close(t);
	// the descriptors built as the calls came, when every packet's header is
	// among them: the kernel stores every field (CGCK_STORE)
	const bool fast = t.txd_ok && t.txd_noip == 0 && !t.txd_fast.empty();
	if (t.txd_ok && !fast)
		txd_spill(t);
	const int n = fast ? (int)t.txd_calls : (int)t.txq.size();
	tx_take(t, f);
	f.pend.seq = 0;
	f.pend.rc = 0;
	f.n = n;
	f.fast = false;
	if (n) {
		cgck_ctx *c = thread_ctx();
		if (!c)
			return -ENODEV;
		int rc;
		if (fast) {
			// The kernel returns each descriptor's two values and the
			// completion writes the fields (tx_write_fast): a ring line
			// the GPU stores into leaves the worker's caches, so the stack's
			// next writes to that slot miss (kernel
			// stores 3.9 against 3.7 us at 256 x 64 B, and 27-55 against 25
			// at 2048).
			const bool kstore = tx_kstore();
			f.d.swap(t.txd_fast);
			f.hs.swap(t.txd_hs);
			f.lo = const_cast<uint8_t *>(t.txd_lo);
			f.stored = kstore;
			f.fast = !kstore;
			if (f.fast)
				f.o.resize(f.d.size());
			const DescSummary sum = {t.txd_max, t.txd_bytes};
			rc = desc_host_post(c, (void *)t.txd_lo, (size_t)(t.txd_hi - t.txd_lo), f.d.data(), f.d.size(),
					    tx_flags(f) | (kstore ? CGCK_STORE : 0u), kstore ? nullptr : f.o.data(), nullptr, nullptr,
					    &f.pend, &sum);
		} else {
			rc = tx_compute(c, f, true);
		}
		if (rc < 0) {
			f.q.clear();
			return rc;
		}
	}
	t.txp_count++;
	return n;
}

extern "C" int cgck_tx_complete(void)
{
	ThreadState &t = tstate();
	if (t.txp_count == 0)
		return 0;
	TxFill &f = t.txp[t.txp_head];
	t.txp_head ^= 1;
	t.txp_count--;
	const int rc = f.pend.seq ? burst_collect(t.ctx, &f.pend) : f.pend.rc;
	if (rc < 0) {
		f.q.clear();
		return rc;
	}
	if (f.stored) { // the kernel wrote them
		f.q.clear();
		return f.n;
	}
	if (f.fast)
		return tx_write_fast(f);
	return tx_write(f);
}

// --------------------------------------------------------------------------
// Toeplitz drop-ins (subr.h:370-371; bodies subr.c:482-502, 506-530)
// --------------------------------------------------------------------------

namespace {

// One toeplitz_hash on the calling thread's context: the data is staged in
// pinned memory, which the kernel reads over the fabric.
uint32_t one_toeplitz(const uint8_t *data, uint32_t cnt, const uint8_t *key, int key_size, uint32_t mask)
{
	cgck_ctx *c = thread_ctx();
	if (!c)
		die("no gfx950 context for the drop-in Toeplitz hash");
	if (grow_host((void **)&c->h_stage, &c->h_stage_cap, cnt + 16) ||
	    grow_host((void **)&c->h_out, &c->h_out_cap, 64))
		die("staging allocation");
	if (cnt)
		memcpy(c->h_stage, data, cnt);
	if (hipSetDevice(c->device) != hipSuccess || rss_prepare(c, key, key_size, cnt, c->stream) != 0)
		die("rss tables");
	RssParams p = {c->h_stage, 1, 0, cnt, mask, c->d_rss_tab, c->h_out};
	hipError_t e = launch_toeplitz(p, c->num_cus, c->stream);
	if (e == hipSuccess)
		e = hipStreamSynchronize(c->stream);
	if (e != hipSuccess) {
		set_err(-EIO, "toeplitz: %s", hipGetErrorString(e));
		die("toeplitz kernel");
	}
	return c->h_out[0];
}

} // namespace

extern "C" uint32_t toeplitz_hash(const unsigned char *data, int cnt, const unsigned char *key, int key_size)
{
	if (cnt > (int)kRssMaxCnt) {
		set_err(-EINVAL, "toeplitz_hash: cnt %d above %u", cnt, kRssMaxCnt);
		die("toeplitz_hash");
	}
	// cnt <= 0: the reference's loop does not run and returns 0 (subr.c:490).
	return one_toeplitz(data, cnt > 0 ? (uint32_t)cnt : 0, key, key_size, 0xffffffffu);
}

extern "C" uint32_t rss_hash4(uint32_t laddr, uint32_t faddr, uint16_t lport, uint16_t fport, unsigned char *key,
			      int key_size)
{
	// subr.c:513-521: faddr, laddr, fport, lport as stored (network order).
	uint8_t d[12];
	memcpy(d + 0, &faddr, 4);
	memcpy(d + 4, &laddr, 4);
	memcpy(d + 8, &fport, 2);
	memcpy(d + 10, &lport, 2);
	return one_toeplitz(d, 12, key, key_size, 0x7Fu); // subr.c:523
}
