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
#include <time.h>

#include <algorithm>
#include <atomic>
#include <vector>

#include "cgck_host.h"

using namespace cgck;

#if CGCK_LAB
extern thread_local double t_lab_post[16]; // cgck_api.cpp: the Poster's phase totals (lab, TSC ticks)
#endif

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

// cgck_rx_begin's burst: its descriptors and the kernel's values and meta
// words (kFlagRx).
struct RxBurst {
	const uint8_t *base = nullptr;
	uint64_t n = 0;
	std::vector<cgck_desc_t> d;
	std::vector<uint32_t> o, m;
};

// The posted (pipelined) windows keep a queue per thread and kind: receive
// bursts (cgck_rx_post) and TX fills (cgck_tx_post), up to kPostQ each,
// opened / completed oldest first.  At most one burst-server request per
// queue is in flight; what is posted while it is in flight waits and goes
// out with everything else posted meanwhile as ONE request once it is back.
// So a loop posting small bursts faster than the GPU answers one (a busy
// worker at a handful of frames per poll) pays one mailbox round trip per
// GPU service time, not per burst, and never waits for the GPU while older
// bursts are still to be processed; a lone burst goes out at once.
constexpr unsigned kPostQ = 64;

// One server request carrying the descriptors of one or more posted items.
struct PostReq {
	std::vector<cgck_desc_t> d;
	std::vector<uint32_t> o, m; // values, meta words (RX)
	BurstPending pend{};
	unsigned items = 0; // posted items it carries, not yet consumed
	bool used = false;  // slot taken (from its send until done with no item left)
	bool done = false;  // o / m hold its values (or rc its failure)
	int rc = 0;
	char msg[192] = {0};
};

// One posted item: a receive burst or a TX fill.  Its n descriptors index
// [base, base + bytes); `own`: no request (nothing to compute, or a staged
// TX fill computed at its post into vals).
struct PostItem {
	const uint8_t *base = nullptr;
	size_t bytes = 0;
	uint32_t flags = 0;
	uint64_t n = 0;
	size_t pkt_bytes = 0; // 16-byte-rounded packet bytes (the server's caps)
	uint32_t max_len = 0;
	std::vector<cgck_desc_t> d;
	std::vector<uint32_t> vals;
	int req = -1;     // request slot, -1: not sent yet
	uint32_t off = 0; // its first descriptor in the request
	bool own = false;
};

// One kind's posted items (receive bursts or TX fills), oldest first; the
// requests that carry them belong to the thread's Poster.
struct PostQueue {
	PostItem it[kPostQ];
	unsigned head = 0, count = 0, sent = 0; // oldest item; items posted; of them sent (oldest first)

	PostItem &at(unsigned k) { return it[(head + k) % kPostQ]; }
	PostItem &oldest() { return it[head]; }
	const PostItem &oldest() const { return it[head]; }
	unsigned next_slot() const { return (head + count) % kPostQ; }
	PostItem &push()
	{
		PostItem &x = it[next_slot()];
		count++;
		x.req = -1;
		x.off = 0;
		x.own = false;
		x.n = 0;
		x.pkt_bytes = 0;
		x.max_len = 0;
		return x;
	}
};

// The thread's two queues and the burst-server requests that carry them.
// One request per kind is in flight; what is posted meanwhile goes out when
// it is back.  When both kinds have items waiting over the same registered
// range, they go out as ONE two-part request (BurstReq.n1: the receive
// frames, then the fill's packets, each with its own flags), so a loop that
// posts a burst and a fill every iteration pays one mailbox round trip for
// both.
enum { kRx = 0, kTx = 1 };

#if CGCK_LAB
// Lab build: where the posted windows' host time goes (tools/txloop split
// mode reads it through cgck_lab_post_times): ns and calls of burst_ready,
// of collect (and of its copy out of the response slot, inside burst_collect)
// and of send.
static inline double lab_ns() { return (double)__builtin_ia32_rdtsc(); } // TSC ticks (lab)
#define LAB_T0(v) const double v = lab_ns()
#define LAB_ADD(i, v) (t_lab_post[2 * (i)] += lab_ns() - (v), t_lab_post[2 * (i) + 1] += 1)
#else
#define LAB_T0(v)
#define LAB_ADD(i, v) ((void)0)
#endif

struct Poster {
	PostQueue q[2];
	// Each live request carries >= 1 unconsumed item, so at most 2 * kPostQ
	// are live at once; a request frees when done with no item left, in any
	// order (one that still holds an old unconsumed fill must not pin the slots
	// of later requests), and send takes the next free slot after the last.
	PostReq rq[2 * kPostQ];
	unsigned rnext = 0, rlive = 0;
	int inflight[2] = {-1, -1}; // the request carrying each kind's sent items (one, when fused)

	bool done(const PostItem &x) const { return x.own || (x.req >= 0 && rq[x.req].done); }
	int rc_of(const PostItem &x) const { return x.own ? 0 : rq[x.req].rc; }
	const char *msg_of(const PostItem &x) const { return x.own ? "" : rq[x.req].msg; }
	const uint32_t *values(const PostItem &x) const { return x.own ? x.vals.data() : rq[x.req].o.data() + x.off; }
	const uint32_t *metas(const PostItem &x) const { return x.own ? nullptr : rq[x.req].m.data() + x.off; }
	int take_slot();
	void release_if_free(int ri);
	bool backlog(const cgck_ctx *c, int kind);
	void bound(cgck_ctx *c, int kind);
	void send(cgck_ctx *c);
	void collect(cgck_ctx *c, int ri);
	void pump(cgck_ctx *c, int kind, bool wait);
	int settle(cgck_ctx *c, int kind, bool wait);
	void pop(int kind);
};

// TX fill bookkeeping beside its PostItem (same slot): the queued fields,
// and for each the value (descriptor) it takes.
struct TxFill {
	std::vector<TxEntry> q;
	std::vector<uint32_t> idx; // entry i's value: values[idx[i]]
	bool fast = false;  // fast form: descriptor k's values, hs[k] its spans
	bool icmp = false;  // holds ICMP messages (their L4 value without the pseudo-header)
	int n = 0;          // the fields it stands for (q is empty in the fast form)
	std::vector<uint32_t> hs;
	uint8_t *lo = nullptr;
};

// cgck_window_stats_n's counters (the first four are cgck_window_stats')
constexpr int kStats = 5;

struct ThreadState {
	cgck_ctx *ctx = nullptr;
	int bind_dev = -1; // cgck_thread_bind's device (-1: $CGCK_DEVICE, default 0)
	// TX window
	bool tx_open = false;
	bool tx_icmp = false; // an ICMP message was queued (icmp_send, ip_icmp.c:68-80)
	std::vector<TxEntry> txq;
	const uint8_t *tx_max = nullptr; // highest header address queued so far
	bool tx_map = false;             // txidx built (the first call below tx_max)
	PtrMap txidx; // (ip << 1 | is_l4) -> txq index
	TxFill txs;       // cgck_tx_flush's batch
	PostItem txs_item;
	TxFill txf[kPostQ]; // the posted fills' bookkeeping, slot for slot with post.q[kTx]
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
	bool rx_span_built = false;
	uintptr_t rx_lo = 0, rx_hi = 0;
	// the last closed RX window's frames (descriptors swapped out of the
	// burst at cgck_rx_end, no copy): a TX-window call queued on one of their
	// headers is counted in stats[4] (the stack verifying a received frame
	// outside an RX window, include/cgck.h); its header addresses are sorted
	// on the first queued call inside the burst's span
	std::vector<cgck_desc_t> last_d;
	const uint8_t *last_base = nullptr;
	bool last_span = false, last_sorted = false;
	uintptr_t last_lo = 0, last_hi = 0;
	std::vector<uintptr_t> last_hdr;
	RxBurst rxs;      // cgck_rx_begin's burst
	Poster post;      // posted bursts (cgck_rx_post) and fills (cgck_tx_post)
	uint64_t rx_served0 = 0; // stats[0] at rx_begin
	uint64_t stats[kStats] = {0, 0, 0, 0, 0};
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
__attribute__((tls_model("initial-exec"))) thread_local uint64_t t_stats_kept[kStats] = {0, 0, 0, 0, 0};
// and its cgck_thread_bind device
__attribute__((tls_model("initial-exec"))) thread_local int t_bind_kept = -1;

ThreadState &tstate()
{
	if (__builtin_expect(!t_st, 0)) {
		t_st = new ThreadState;
		memcpy(t_st->stats, t_stats_kept, sizeof(t_stats_kept));
		t_st->bind_dev = t_bind_kept;
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

// [rx_lo, rx_hi): the bytes the burst's frames span, computed on the first
// call the cursor probe does not answer (most bursts never need it).
__attribute__((noinline)) void rx_span(ThreadState &t)
{
	uintptr_t lo = UINTPTR_MAX, hi = 0;
	for (size_t i = 0; i < t.rx_n; i++) {
		const uintptr_t a = (uintptr_t)(t.rx_base + t.rxd[i].frame_off);
		const uintptr_t e = a + t.rxd[i].l3_off + t.rxd[i].ip_len;
		lo = a < lo ? a : lo;
		hi = e > hi ? e : hi;
	}
	t.rx_lo = lo;
	t.rx_hi = hi;
	t.rx_span_built = true;
}

inline bool rx_in_span(ThreadState &t, const uint8_t *p)
{
	if (!t.rx_span_built)
		rx_span(t);
	return (uintptr_t)p >= t.rx_lo && (uintptr_t)p < t.rx_hi;
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
	// Off the cursor: a call outside the burst's address span (a reply the
	// stack builds in a transmit slot while the window is open) is no frame
	// of the burst, and needs neither the map nor rx_owns
	if (!rx_in_span(t, p))
		return false;
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
	if (!rx_in_span(t, p))
		return false;
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

// A TX-window call queued on the header of a frame of the last closed RX
// burst (stats[4]): a received frame verified outside an RX window looks like
// a transmit call and is queued, so the stack got 0 for it (include/cgck.h).
// A transport that reuses a received frame for a reply in the same iteration
// counts here too; the counter names the frames to look at, it drops nothing.
__attribute__((noinline)) void tx_note_last_rx_slow(ThreadState &t, const uint8_t *ip)
{
	const size_t n = t.last_d.size();
	if (!t.last_span) {
		uintptr_t lo = UINTPTR_MAX, hi = 0;
		for (size_t i = 0; i < n; i++) {
			const uintptr_t a = (uintptr_t)(t.last_base + t.last_d[i].frame_off + t.last_d[i].l3_off);
			lo = a < lo ? a : lo;
			hi = a + 1 > hi ? a + 1 : hi;
		}
		t.last_lo = lo;
		t.last_hi = hi;
		t.last_span = true;
	}
	const uintptr_t p = (uintptr_t)ip;
	if (p < t.last_lo || p >= t.last_hi)
		return;
	if (!t.last_sorted) {
		t.last_hdr.resize(n);
		for (size_t i = 0; i < n; i++)
			t.last_hdr[i] = (uintptr_t)(t.last_base + t.last_d[i].frame_off + t.last_d[i].l3_off);
		std::sort(t.last_hdr.begin(), t.last_hdr.end());
		t.last_sorted = true;
	}
	t.stats[4] += std::binary_search(t.last_hdr.begin(), t.last_hdr.end(), p);
}

inline void tx_note_last_rx(ThreadState &t, const uint8_t *ip)
{
	if (__builtin_expect(!t.last_d.empty(), 0))
		tx_note_last_rx_slow(t, ip);
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
		const int dev = t.bind_dev >= 0 ? t.bind_dev : e ? atoi(e) : 0;
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

// The device of this thread's drop-in context, chosen before its first use
// (con-gen's thread_init: the worker's RSS queue id modulo the devices).
extern "C" int cgck_thread_bind(int device)
{
	const int nd = cgck_device_count();
	if (nd < 0)
		return nd;
	if (device < 0 || device >= nd)
		return set_err(-EINVAL, "cgck_thread_bind: device %d of %d", device, nd);
	ThreadState &t = tstate();
	if (t.ctx && t.ctx->device != device)
		return set_err(-EBUSY, "cgck_thread_bind: this thread's context is already on device %d "
				       "(cgck_thread_release first)", t.ctx->device);
	t.bind_dev = device;
	return 0;
}

extern "C" int cgck_thread_device(void)
{
	const ThreadState *t = t_st;
	if (t && t->ctx)
		return t->ctx->device;
	if (t && t->bind_dev >= 0)
		return t->bind_dev;
	const char *e = getenv("CGCK_DEVICE");
	return e ? atoi(e) : 0;
}

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
	t_bind_kept = t->bind_dev;
	delete t;
	t_st = nullptr;
	return 0;
}

extern "C" int cgck_window_stats(uint64_t stats[4])
{
	if (!stats)
		return set_err(-EINVAL, "cgck_window_stats: NULL");
	memcpy(stats, t_st ? t_st->stats : t_stats_kept, 4 * sizeof(uint64_t));
	return 0;
}

extern "C" int cgck_window_stats_n(uint64_t *stats, int n)
{
	if (!stats || n < 0)
		return set_err(-EINVAL, "cgck_window_stats_n: NULL or negative count");
	const int k = n < kStats ? n : kStats;
	memcpy(stats, t_st ? t_st->stats : t_stats_kept, (size_t)k * sizeof(uint64_t));
	return kStats;
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
				tx_note_last_rx(t, b);
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
					tx_note_last_rx(t, ip);
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
				tx_note_last_rx(t, ip);
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

// The unsent items of one kind that go out together: as many as share the
// first one's range and flags and fit what is left of the server's caps
// (without a server the request is a launch, computed at once).  Items
// computed at their post are stepped over.
struct Group {
	unsigned s = 0, e = 0; // items [s, e) of the queue (from its oldest)
	uint64_t n = 0;        // descriptors
	size_t pb = 0;
	uint32_t ml = 0;
	const PostItem *f = nullptr;
};

static Group gather(PostQueue &q, uint64_t cap_n, size_t cap_b)
{
	Group g;
	while (q.sent < q.count && q.at(q.sent).own)
		q.sent++;
	g.s = g.e = q.sent;
	if (q.sent == q.count)
		return g;
	g.f = &q.at(q.sent);
	for (unsigned k = q.sent; k < q.count; k++) {
		const PostItem &x = q.at(k);
		if (x.own || x.base != g.f->base || x.bytes != g.f->bytes || x.flags != g.f->flags)
			break;
		if (k > q.sent && (g.n + x.n > cap_n || g.pb + x.pkt_bytes > cap_b))
			break;
		g.n += x.n;
		g.pb += x.pkt_bytes;
		g.ml = x.max_len > g.ml ? x.max_len : g.ml;
		g.e = k + 1;
	}
	return g;
}

// A free request slot.  Live requests never exceed live items (<= 2 * kPostQ),
// so one is always free when an item waits to be sent.
int Poster::take_slot()
{
	for (unsigned k = 0; k < 2 * kPostQ; k++) {
		const unsigned ri = (rnext + k) % (2 * kPostQ);
		if (!rq[ri].used) {
			rq[ri].used = true;
			rnext = (ri + 1) % (2 * kPostQ);
			rlive++;
			return (int)ri;
		}
	}
	return -1;
}

void Poster::release_if_free(int ri)
{
	PostReq &r = rq[ri];
	if (r.used && r.done && r.items == 0) {
		r.used = false;
		rlive--;
	}
}

// The latency bound of the coalesced queues.  While a
// kind's request is in flight, what is posted meanwhile waits and goes out
// together when it is back; a loop that posts faster than the GPU serves (a
// burst of 2048 frames every few us) would otherwise queue up to kPostQ
// requests' worth behind it — 48 bursts, 1.1 ms from post to verdict at 2048
// frames (profiles/r05/final/table_64.txt).  Only one request per kind is
// ever in flight, so a deeper queue buys no GPU throughput: once the unsent
// items hold more than one server request can carry (max_pkts frames or
// max_bytes), the post waits for the request in flight and sends the next
// one, so a posted item is at most ~two service times from its values.
// Small bursts coalesce as before (64 bursts of up to 32 frames fit one
// request).
bool Poster::backlog(const cgck_ctx *c, int kind)
{
	if (!c->bbox || inflight[kind] < 0)
		return false;
	const PostQueue &qq = q[kind];
	uint64_t n = 0;
	size_t b = 0;
	for (unsigned k = qq.sent; k < qq.count; k++) {
		const PostItem &x = qq.it[(qq.head + k) % kPostQ];
		if (x.own)
			continue;
		n += x.n;
		b += x.pkt_bytes;
	}
	return n > c->bmax || b > c->bmax_bytes;
}

void Poster::bound(cgck_ctx *c, int kind)
{
	for (int k = 0; k < 4 && backlog(c, kind); k++)
		pump(c, kind, true);
}

// Send what each kind with nothing in flight has waiting: both kinds as one
// two-part request when they share the range (the receive frames first, so
// their meta words come back too), else one request each.
void Poster::send(cgck_ctx *c)
{
	const uint64_t cap_n = c->bbox ? c->bmax : UINT64_MAX;
	const size_t cap_b = c->bbox ? c->bmax_bytes : SIZE_MAX;
	Group g[2];
	for (int k = 0; k < 2; k++)
		if (inflight[k] < 0)
			g[k] = gather(q[k], cap_n, cap_b);
	// one request when both fit the server together (else one each)
	const bool fuse = g[kRx].f && g[kTx].f && c->bbox && g[kRx].f->base == g[kTx].f->base &&
			  g[kRx].f->bytes == g[kTx].f->bytes && g[kRx].n + g[kTx].n <= cap_n &&
			  g[kRx].pb + g[kTx].pb <= cap_b;
	for (int k = 0; k < 2; k++) {
		if (!g[k].f || (fuse && k == kTx))
			continue;
		const int parts = fuse ? 2 : 1;
		const int ri = take_slot();
		if (ri < 0) // cannot happen (see take_slot); leave the items unsent
			die("cgck posted windows: no free request slot");
		PostReq &r = rq[ri];
		r.d.clear();
		r.items = 0;
		for (int pk = k; pk < k + parts; pk++) {
			PostQueue &qq = q[pk];
			for (unsigned j = g[pk].s; j < g[pk].e; j++) {
				PostItem &x = qq.at(j);
				if (x.own)
					continue;
				x.req = ri;
				x.off = (uint32_t)r.d.size();
				r.d.insert(r.d.end(), x.d.begin(), x.d.end());
				r.items++;
			}
			qq.sent = g[pk].e;
			inflight[pk] = ri;
		}
		const uint64_t n = r.d.size();
		r.o.resize(n);
		r.m.resize(n);
		r.done = false;
		r.rc = 0;
		r.msg[0] = 0;
		const DescSummary sum = {g[k].ml > g[kTx].ml || !fuse ? g[k].ml : g[kTx].ml,
					 g[k].pb + (fuse ? g[kTx].pb : 0)};
		const DescSplit split = {(uint32_t)g[kRx].n, fuse ? g[kTx].f->flags : 0u};
		const int rc = desc_host_post(c, const_cast<uint8_t *>(g[k].f->base), g[k].f->bytes, r.d.data(), n,
					      g[k].f->flags, r.o.data(), nullptr, k == kRx ? r.m.data() : nullptr, &r.pend,
					      &sum, fuse ? &split : nullptr);
		if (rc < 0) {
			r.rc = rc;
			snprintf(r.msg, sizeof(r.msg), "%s", err_text());
			r.done = true;
		} else if (rc == 0) {
			r.done = true;
		}
		if (r.done)
			for (int pk = k; pk < k + parts; pk++)
				inflight[pk] = -1;
	}
}

// Collect request ri (waiting for it if it is not back).
void Poster::collect(cgck_ctx *c, int ri)
{
	PostReq &r = rq[ri];
	LAB_T0(t0);
	r.rc = r.pend.seq ? burst_collect(c, &r.pend) : r.pend.rc;
	LAB_ADD(1, t0);
	if (r.rc)
		snprintf(r.msg, sizeof(r.msg), "%s", err_text());
	r.done = true;
	for (int k = 0; k < 2; k++)
		if (inflight[k] == ri)
			inflight[k] = -1;
}

// Collect the requests in flight that are back (wait: also `kind`'s, once
// it is back), then send what was posted meanwhile.
void Poster::pump(cgck_ctx *c, int kind, bool wait)
{
	for (int k = 0; k < 2; k++) {
		const int ri = inflight[k];
		bool go = ri >= 0 && wait && k == kind;
		if (ri >= 0 && !go) {
			LAB_T0(t0);
			go = burst_ready(c, &rq[ri].pend);
			LAB_ADD(0, t0);
		}
		if (go)
			collect(c, ri);
	}
	// only a kind with nothing in flight sends (send gathers for no other)
	if ((inflight[kRx] < 0 && q[kRx].sent < q[kRx].count) || (inflight[kTx] < 0 && q[kTx].sent < q[kTx].count)) {
		LAB_T0(t0);
		send(c);
		LAB_ADD(3, t0);
	}
}

// Are the oldest item's values in (1), or not yet (0)?  wait: until they are.
int Poster::settle(cgck_ctx *c, int kind, bool wait)
{
	pump(c, kind, false);
	while (!done(q[kind].oldest())) {
		if (!wait)
			return 0;
		pump(c, kind, true);
	}
	return 1;
}

// The oldest item of a kind consumed; requests all of whose items are
// consumed free, oldest first.
void Poster::pop(int kind)
{
	PostQueue &qq = q[kind];
	PostItem &x = qq.oldest();
	const int ri = x.req;
	if (ri >= 0)
		rq[ri].items--;
	qq.head = (qq.head + 1) % kPostQ;
	qq.count--;
	if (qq.sent)
		qq.sent--;
	if (ri >= 0)
		release_if_free(ri);
}

// Open the window over a computed burst; returns the frames it answers for.
int rx_open_on(ThreadState &t, const uint8_t *base, uint64_t n, const cgck_desc_t *d, const uint32_t *o,
	       const uint32_t *m, bool posted)
{
	uint64_t k = 0;
	for (uint64_t i = 0; i < n; i++)
		k += m[i] != 0;
	t.rxd = d;
	t.rxo = o;
	t.rxm = m;
	t.rx_base = base;
	t.rx_n = n;
	t.rx_cur = 0;
	t.rx_map = false;
	t.rx_iv_built = false;
	t.rx_span_built = false;
	t.rx_open = true;
	t.rx_posted = posted;
	t.rx_served0 = t.stats[0];
	return (int)k;
}

int rx_check(const void *base, const cgck_desc_t *desc, uint64_t n, const char *who)
{
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
	int rc = rx_check(base, desc, n, "cgck_rx_begin");
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
	RxBurst &r = t.rxs;
	r.base = (const uint8_t *)base;
	r.n = n;
	r.d.assign(desc, desc + n);
	r.o.resize(n ? n : 1);
	r.m.resize(n ? n : 1);
	if (n && (rc = desc_host(c, base, bytes, r.d.data(), n, kRxFlags, r.o.data(), nullptr, r.m.data()))) {
		char msg[256];
		snprintf(msg, sizeof(msg), "%s", err_text());
		return set_err(rc, "cgck_rx_begin: %s", msg);
	}
	return rx_open_on(t, r.base, n, r.d.data(), r.o.data(), r.m.data(), false);
}

// Pipelined form: post burst k and return; the window over it opens at a
// later cgck_rx_begin_posted, while the stack has worked on older bursts.
// The descriptors are checked here, so a bad one fails its own post.
extern "C" int cgck_rx_post(void *base, size_t bytes, const cgck_desc_t *desc, uint64_t n)
{
	ThreadState &t = tstate();
	PostQueue &q = t.post.q[kRx];
	if (q.count == kPostQ)
		return set_err(-EBUSY, "cgck_rx_post: %u bursts already posted and not yet opened", kPostQ);
	int rc = rx_check(base, desc, n, "cgck_rx_post");
	if (rc)
		return rc;
	cgck_ctx *c = thread_ctx();
	if (!c)
		return -ENODEV;
	size_t pb = 0;
	uint32_t ml = 0;
	for (uint64_t i = 0; i < n; i++) {
		const uint64_t end = desc[i].frame_off + desc[i].l3_off + desc[i].ip_len;
		if (end > bytes || end < desc[i].frame_off)
			return set_err(-EINVAL, "cgck_rx_post: descriptor %llu reaches past the %zu bytes given",
				       (unsigned long long)i, bytes);
		ml = desc[i].ip_len > ml ? desc[i].ip_len : ml;
		pb += ((size_t)desc[i].ip_len + 15) & ~(size_t)15;
	}
	PostItem &x = q.push();
	x.base = (const uint8_t *)base;
	x.bytes = bytes;
	x.flags = kRxFlags;
	x.n = n;
	x.d.assign(desc, desc + n);
	x.pkt_bytes = pb;
	x.max_len = ml;
	x.own = n == 0;
	x.vals.clear();
	t.post.pump(c, kRx, false);
	t.post.bound(c, kRx);
	return (int)n;
}

extern "C" int cgck_rx_begin_posted(void)
{
	ThreadState &t = tstate();
	Poster &P = t.post;
	if (t.rx_open)
		return set_err(-EBUSY, "cgck_rx_begin_posted: an RX window is already open on this thread");
	if (P.q[kRx].count == 0)
		return set_err(-ENOENT, "cgck_rx_begin_posted: no burst posted");
	P.settle(t.ctx, kRx, true);
	const PostItem &x = P.q[kRx].oldest();
	if (const int rc = P.rc_of(x)) {
		char msg[200];
		snprintf(msg, sizeof(msg), "%s", P.msg_of(x));
		P.pop(kRx);
		return set_err(rc, "cgck_rx_begin_posted: %s", msg);
	}
	static const uint32_t none = 0;
	return rx_open_on(t, x.base, x.n, x.d.data(), x.n ? P.values(x) : &none, x.n ? P.metas(x) : &none, true);
}

// The drain rule's two questions (include/cgck.h): is a burst still posted,
// and would opening the oldest one wait for the GPU?
#if CGCK_LAB
// Lab: the Poster's phase totals (TSC ticks, calls) since the last call, zeroed.
extern "C" void cgck_lab_post_times(double out[16])
{
	memcpy(out, t_lab_post, sizeof(t_lab_post));
	memset(t_lab_post, 0, sizeof(t_lab_post));
}
#endif

extern "C" int cgck_rx_pending(void)
{
	const ThreadState *t = t_st;
	return t ? (int)t->post.q[kRx].count : 0;
}

extern "C" int cgck_rx_ready(void)
{
	ThreadState *t = t_st;
	if (!t || t->post.q[kRx].count == 0)
		return set_err(-ENOENT, "cgck_rx_ready: no burst posted");
	return t->post.settle(t->ctx, kRx, false);
}

extern "C" int cgck_rx_end(void)
{
	ThreadState &t = tstate();
	if (!t.rx_open)
		return set_err(-EINVAL, "cgck_rx_end: no open RX window on this thread");
	t.rx_open = false;
	t.rx_map = false;
	// keep the closed burst's frames for stats[4] (a swap, no copy)
	if (t.rx_posted)
		std::swap(t.last_d, t.post.q[kRx].oldest().d);
	else
		std::swap(t.last_d, t.rxs.d);
	t.last_base = t.rx_base;
	t.last_span = t.last_sorted = false;
	t.rx_n = 0;
	if (t.rx_posted) {
		t.rx_posted = false;
		t.post.pop(kRx);
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

// Both kinds in one batch (kTxFlags, cgck_internal.h): IP entries ask for
// the header checksum, L4 entries for the segment checksum; both read their
// fields as zero, as the reference's callers have just stored them
// (ip_output.c:61, tcp_subr.c:75 / gbtcp/tcp.c:426,436).

// A fill with ICMP messages also asks for their values without the
// pseudo-header (kFlagL4Auto: by ip_p, as the RX window does); TCP and UDP
// keep it.  Only then, because the lane-per-packet kernels take no
// kFlagL4Auto and the group kernel is slower on small frames.
inline uint32_t tx_flags(const TxFill &f) { return kTxFlags | (f.icmp ? kFlagL4Auto : 0u); }

// Describe the entries of f.q for the kernel, into x.  When every entry lies
// in one registered range (the transport's pool) the batch is described in
// place, as cgck_desc_host of that range (returns 1: x is to be computed);
// otherwise each region is staged 16-byte aligned in pinned memory and
// computed at once into x.vals (returns 0).  f.idx[i] is entry i's value.
int tx_build(cgck_ctx *c, TxFill &f, PostItem &x)
{
	const std::vector<TxEntry> &q = f.q;
	const uint64_t n = q.size();
	x.flags = tx_flags(f);
	HIP_TRY(hipSetDevice(c->device));
	RegRange reg{nullptr, nullptr, nullptr};
	bool inplace = reg_find(q[0].ip, q[0].span, &reg);
	for (uint64_t i = 1; inplace && i < n; i++)
		inplace = q[i].ip >= reg.lo && q[i].ip + q[i].span <= reg.hi;
	// One descriptor per packet: a packet's header entry and its segment
	// entry (queued one after the other by the finalisers, ip_output.c:61-64
	// after tcp_output.c:416-418) share it — it covers the segment, and the
	// kernel returns both the header checksum (over ip_hl * 4 bytes, which
	// the queue checked equals the header call's length) and the segment's
	// L4 checksum from one read of the frame.
	f.idx.resize(n);
	if (inplace) {
		x.d.resize(n);
		uint64_t m = 0;
		for (uint64_t i = 0; i < n; i++) {
			if (i > 0 && q[i].ip == q[i - 1].ip && (q[i].fo < 0) != (q[i - 1].fo < 0) && f.idx[i - 1] == m - 1 &&
			    (i < 2 || f.idx[i - 2] != m - 1)) {
				f.idx[i] = (uint32_t)(m - 1);
				if (q[i].span > x.d[m - 1].ip_len)
					x.d[m - 1].ip_len = (uint16_t)q[i].span;
				continue;
			}
			f.idx[i] = (uint32_t)m;
			x.d[m].frame_off = (uint64_t)(q[i].ip - reg.lo);
			x.d[m].l3_off = 0;
			x.d[m].ip_len = (uint16_t)q[i].span;
			m++;
		}
		x.d.resize(m);
		x.base = reg.lo;
		x.bytes = (size_t)(reg.hi - reg.lo);
		x.n = m;
		x.pkt_bytes = 0;
		x.max_len = 0;
		for (const cgck_desc_t &e : x.d) {
			x.pkt_bytes += ((size_t)e.ip_len + 15) & ~(size_t)15;
			x.max_len = e.ip_len > x.max_len ? e.ip_len : x.max_len;
		}
		x.own = false;
		return 1;
	}
	for (uint64_t i = 0; i < n; i++)
		f.idx[i] = (uint32_t)i;
	size_t bytes = 0; // staged bytes
	for (const TxEntry &e : q)
		bytes += (e.span + 15) & ~(size_t)15;
	const size_t d_off = (bytes + 15) & ~(size_t)15;
	const size_t o_off = (d_off + 12 * n + 15) & ~(size_t)15;
	int rc;
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
	KParams p = {h, d, n, 0, 0, 0, x.flags, o, nullptr, nullptr, 0, nullptr};
	if ((rc = run(c, p, 1500, c->stream)))
		return rc;
	HIP_TRY(CGCK_SYNC(c->stream));
	x.vals.assign(o, o + n);
	x.d.clear();
	x.n = 0;
	x.own = true;
	return 0;
}

// Write every queued field from the computed values; returns their count.
int tx_write(TxFill &f, const uint32_t *vals)
{
	const std::vector<TxEntry> &q = f.q;
	const uint64_t n = q.size();
	for (uint64_t i = 0; i < n; i++) {
		uint16_t v;
		uint8_t *dst;
		const uint32_t r = vals[f.idx[i]];
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

// The fields of a fill in the fast form, from descriptor k's values: its
// header's (ip+10) when the header was queued, its segment's when the
// segment was (at ip_hl * 4 + 16 for TCP, + 6 for UDP, + 2 for ICMP, read
// from the packet as the call read them).
int tx_write_fast(const TxFill &f, const PostItem &x, const uint32_t *vals)
{
	for (size_t k = 0; k < x.n; k++) {
		uint8_t *ip = f.lo + x.d[k].frame_off;
		const uint32_t r = vals[k], hs = f.hs[k];
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

// Close the window into f and x: the fast form's descriptors as they are
// (every packet's header among them), else the entry queue (returns 1), or
// nothing queued (0).
int tx_take(ThreadState &t, TxFill &f, PostItem &x)
{
	txd_close(t);
	const bool fast = t.txd_ok && t.txd_noip == 0 && !t.txd_fast.empty();
	if (t.txd_ok && !fast)
		txd_spill(t);
	t.tx_open = false;
	t.tx_map = false;
	f.icmp = t.tx_icmp;
	f.fast = fast;
	f.q.swap(t.txq);
	t.txq.clear();
	x.own = false;
	x.vals.clear();
	if (fast) {
		x.d.swap(t.txd_fast);
		f.hs.swap(t.txd_hs);
		f.lo = const_cast<uint8_t *>(t.txd_lo);
		f.n = (int)t.txd_calls;
		x.base = t.txd_lo;
		x.bytes = (size_t)(t.txd_hi - t.txd_lo);
		x.n = x.d.size();
		x.pkt_bytes = t.txd_bytes;
		x.max_len = t.txd_max;
		x.flags = tx_flags(f);
		return 1;
	}
	f.n = (int)f.q.size();
	x.n = 0;
	return f.n ? 1 : 0;
}

} // namespace

extern "C" int cgck_tx_flush(void)
{
	ThreadState &t = tstate();
	if (!t.tx_open)
		return set_err(-EINVAL, "cgck_tx_flush: no open window on this thread");
	TxFill &f = t.txs;
	PostItem &x = t.txs_item;
	if (!tx_take(t, f, x))
		return 0;
	cgck_ctx *c = thread_ctx();
	if (!c)
		return -ENODEV;
	int rc = f.fast ? 1 : tx_build(c, f, x);
	if (rc == 1) {
		// in place: one request (or launch) over the pool, waited for here
		x.vals.resize(x.n);
		BurstPending pend{};
		const DescSummary sum = {x.max_len, x.pkt_bytes};
		rc = desc_host_post(c, const_cast<uint8_t *>(x.base), x.bytes, x.d.data(), x.n, x.flags, x.vals.data(),
				    nullptr, nullptr, &pend, &sum);
		if (rc >= 0)
			rc = pend.seq ? burst_collect(c, &pend) : pend.rc;
	}
	if (rc < 0) {
		f.q.clear();
		return rc;
	}
	return f.fast ? tx_write_fast(f, x, x.vals.data()) : tx_write(f, x.vals.data());
}

// Pipelined form: post the window's fill and return; cgck_tx_complete
// (before the transport hands these slots to the NIC) waits for it and
// writes the fields.  Fills posted while an earlier one is still on the
// GPU go out together once it is back (PostQueue).
extern "C" int cgck_tx_post(void)
{
	ThreadState &t = tstate();
	if (!t.tx_open)
		return set_err(-EINVAL, "cgck_tx_post: no open window on this thread");
	PostQueue &q = t.post.q[kTx];
	int old_rc = 0;
	char old_msg[200] = {0};
	if (q.count == kPostQ) {
		// The queue is full: the oldest fill completes first (its fields
		// are written now, before the kick that was to wait for them —
		// final values either way), so no queued field is dropped.
		// A failed completion still frees the oldest slot: this window is
		// posted regardless (its calls were answered 0, so dropping it would
		// send zero checksums), and the oldest fill's error is returned
		// after the post (include/cgck.h).
		old_rc = cgck_tx_complete();
		if (old_rc < 0)
			snprintf(old_msg, sizeof(old_msg), "%s", err_text());
	}
	cgck_ctx *c = thread_ctx();
	if (!c)
		return -ENODEV;
	TxFill &f = t.txf[q.next_slot()];
	PostItem &x = q.push();
#if CGCK_LAB
	struct timespec lt[5];
	clock_gettime(CLOCK_MONOTONIC, &lt[0]);
#define LAB_TP(i) clock_gettime(CLOCK_MONOTONIC, &lt[i])
#else
#define LAB_TP(i) ((void)0)
#endif
	int rc = tx_take(t, f, x);
	LAB_TP(1);
	if (rc == 0) {
		x.own = true; // nothing queued: complete as it stands
	} else if (!f.fast && (rc = tx_build(c, f, x)) < 0) {
		// computed at once and failed: the fill leaves the queue unwritten
		q.count--;
		f.q.clear();
		return rc;
	}
	LAB_TP(2);
	t.post.pump(c, kTx, false);
	LAB_TP(3);
	t.post.bound(c, kTx);
	LAB_TP(4);
#if CGCK_LAB
	auto ms = [&](int i) { return (lt[i].tv_sec - lt[i - 1].tv_sec) * 1e3 + (lt[i].tv_nsec - lt[i - 1].tv_nsec) * 1e-6; };
	if (ms(1) + ms(2) + ms(3) + ms(4) > 20)
		fprintf(stderr, "cgck lab: tx_post %.1f ms: take %.3f build %.3f (fast %d, own %d, n %llu) pump %.3f bound %.3f\n",
			ms(1) + ms(2) + ms(3) + ms(4), ms(1), ms(2), (int)f.fast, (int)x.own, (unsigned long long)x.n, ms(3),
			ms(4));
#endif
#undef LAB_TP
	if (old_rc < 0)
		return set_err(old_rc, "cgck_tx_post: this window was posted, but completing the oldest fill failed "
				       "(its fields are not written): %s", old_msg);
	return f.n;
}

extern "C" int cgck_tx_complete(void)
{
	ThreadState &t = tstate();
	Poster &P = t.post;
	PostQueue &q = P.q[kTx];
	if (q.count == 0)
		return 0;
	P.settle(t.ctx, kTx, true);
	const PostItem &x = q.oldest();
	TxFill &f = t.txf[q.head];
	if (const int rc = P.rc_of(x)) {
		char msg[200];
		snprintf(msg, sizeof(msg), "%s", P.msg_of(x));
		f.q.clear();
		P.pop(kTx);
		return set_err(rc, "cgck_tx_complete: %s", msg);
	}
	const int n = f.n == 0 ? 0 : f.fast ? tx_write_fast(f, x, P.values(x)) : tx_write(f, P.values(x));
	P.pop(kTx);
	return n;
}

extern "C" int cgck_tx_pending(void)
{
	const ThreadState *t = t_st;
	return t ? (int)t->post.q[kTx].count : 0;
}

extern "C" int cgck_tx_ready(void)
{
	ThreadState *t = t_st;
	if (!t || t->post.q[kTx].count == 0)
		return set_err(-ENOENT, "cgck_tx_ready: no fill posted");
	return t->post.settle(t->ctx, kTx, false);
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
		e = CGCK_SYNC(c->stream);
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
