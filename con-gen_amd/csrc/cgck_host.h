// cgck_host.h — host-side internals shared by cgck_api.cpp (contexts,
// batches, rings, RSS, plumbing) and cgck_dropin.cpp (the drop-in symbols and
// the per-thread RX / TX windows).  Not part of the C-ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <stddef.h>
#include <stdint.h>

#include <atomic>

#include "cgck_internal.h"

namespace cgck {
// A request left posted on the burst server (desc_host_post): where its
// outputs go when it is collected (burst_collect) and its result.
struct BurstPending {
	uint32_t seq; // 0: not pending
	uint32_t n;
	uint64_t range;
	uint32_t *out, *meta;
	uint8_t *verdict;
	int rc;
};
} // namespace cgck

struct cgck_ctx {
	int device;
	int num_cus;
	hipStream_t stream;
	uint32_t desc_len_hint;
	uint32_t desc_layout; // CGCK_LAYOUT_*
	int family; // kernel family: 0 auto, 1 group, 2 lane-per-packet ($CGCK_KERNEL)
	const char *last_kernel; // cgck_ctx_last_kernel
	// pinned host staging (drop-in calls, deferred TX)
	uint8_t *h_stage;
	size_t h_stage_cap;
	uint32_t *h_out;
	size_t h_out_cap;
	// device scratch (host-resident batches)
	uint8_t *d_bytes;
	size_t d_bytes_cap;
	uint8_t *d_aux; // descriptors | out | verdict
	size_t d_aux_cap;
	void *d_zero; // kZeroBytes zero bytes (KParams.zero)
	// Toeplitz byte tables of the last key used (cgck_rss.hip)
	uint32_t *d_rss_tab;
	size_t d_rss_tab_cap;
	uint32_t *h_rss_tab; // host copy (malloc)
	size_t h_rss_tab_cap;
	uint8_t *rss_key; // the key the tables were built from (malloc)
	int rss_key_len;
	uint32_t rss_cnt;
	bool rss_valid;
	void *rss_users; // RssUsers (cgck_api.cpp): one event per stream that read d_rss_tab
	// dst-cache scratch: control words + look-back status (zeroed per launch)
	uint8_t *d_dst;
	size_t d_dst_cap;
	// burst server (cgck_burst_open): mailbox, request block and outputs in
	// host-coherent pinned memory, the block's device copy in scratch
	cgck::BurstBox *bbox; // nullptr: closed
	uint8_t *bstage;      // request block: [BurstReq | descriptors | packet bytes]
	size_t bstage_cap;
	uint8_t *bstage_dev;        // device view of bstage
	cgck::BurstBox *bbox_dev;   // device view of bbox
	uint8_t *bresp;             // a request's outputs, packed by its n (burst_meta_off / burst_ver_off)
	uint8_t *bresp_dev;
	uint8_t *bscratch;          // device: the server's copy of the block (bstage_cap bytes)
	uint64_t *brelay;           // device, uncached: the leader's relay word
	uint32_t bmax;              // packets per request
	size_t bmax_bytes;          // packet bytes per request (cgck_burst_open's max_bytes)
	uint32_t bwgs;              // workgroups of the server (K)
	uint32_t bper;              // packets per workgroup of a wide request
	uint32_t bbad;              // bbox->bad_req as last seen
	uint32_t bseq;              // the last request posted
	uint32_t bdone;             // the last request known complete (a relaunch serves the ones after it)
	cgck::BurstPending *bslot[2]; // a posted request not yet collected, per slot
	uint32_t bbusy;             // the owner thread is inside a request (MapGuard, cgck_api.cpp)
	// device memory the host writes through the large BAR (nullptr: none, the
	// mailbox words are bbox->req): the two mailbox words the leader polls,
	// then two kBurstFirst request slots for small blocks
	uint64_t *bdoor;
	uint8_t *bvblk;
	bool bnext_vram;            // the block burst_slot_free handed out is a bvblk slot
	uint64_t breq[2];           // the last mailbox word posted per slot (host copy)
	hipStream_t bstream; // the server's own stream (it stays resident)
};

// Library-internal: hidden, so calls between the library's own files are
// direct (no PLT hop on the drop-in symbols' per-call path, e.g. reg_find).
#pragma GCC visibility push(hidden)
namespace cgck {

// hipStreamSynchronize; the lab build reports a synchronisation that takes
// more than 20 ms, with where it was called (a loop stall's diagnosis).
#if CGCK_LAB
hipError_t lab_sync(const char *where, hipStream_t st);
#define CGCK_STR2(x) #x
#define CGCK_STR(x) CGCK_STR2(x)
#define CGCK_SYNC(st) ::cgck::lab_sync(__FILE__ ":" CGCK_STR(__LINE__), st)
#else
#define CGCK_SYNC(st) hipStreamSynchronize(st)
#endif

// Thread-local error text (cgck_last_error); returns `code`.
int set_err(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
const char *err_text();

#define HIP_TRY(expr)                                                                     \
	do {                                                                              \
		hipError_t e_ = (expr);                                                   \
		if (e_ != hipSuccess)                                                     \
			return ::cgck::set_err(-EIO, "%s: %s", #expr, hipGetErrorString(e_)); \
	} while (0)

int grow_host(void **p, size_t *cap, size_t need);
int grow_dev(void **p, size_t *cap, size_t need);

// One checksum launch on the context (KParams.zero filled in); records the
// kernel's name in c->last_kernel.
int run(cgck_ctx *c, const KParams &p, uint32_t len_hint, hipStream_t st);

// cgck_desc_host without the public flag check (internal flags allowed).
// meta: kFlagRx's per-packet words (nullptr otherwise).
int desc_host(cgck_ctx *c, void *base, size_t bytes, const cgck_desc_t *desc, uint64_t n, uint32_t flags,
	      uint32_t *out, uint8_t *verdict, uint32_t *meta = nullptr);
// The same, left posted when the burst server takes it: returns 1 and *pend
// records the request (burst_collect waits for it and copies its outputs to
// out / verdict / meta, which must stay valid until then); 0 when it was
// computed at once (no server, or it does not fit); a negative errno.  A
// later request on the context that needs the slot collects it first.
// sum (optional): the longest ip_len and the 16-byte-rounded packet bytes of
// descriptors the library built itself inside [base, base + bytes), so the
// per-descriptor check is skipped.
struct DescSummary {
	uint32_t max_len;
	size_t pkt_bytes;
};
// A request in two parts: descriptors [n1, n) take flags2 (BurstReq.n1).
struct DescSplit {
	uint32_t n1, flags2;
};
int desc_host_post(cgck_ctx *c, void *base, size_t bytes, const cgck_desc_t *desc, uint64_t n, uint32_t flags,
		   uint32_t *out, uint8_t *verdict, uint32_t *meta, BurstPending *pend,
		   const DescSummary *sum = nullptr, const DescSplit *split = nullptr);
int burst_collect(cgck_ctx *c, BurstPending *pend);
// Without waiting: is the posted request's every slice served (1), or not
// yet (0)?  A request that was computed at once (seq 0) is ready.
int burst_ready(cgck_ctx *c, const BurstPending *pend);

// Staging path of one region for the drop-in symbols (burst server when open,
// else a launch on the context stream and a synchronisation).
int one_region(cgck_ctx *c, const void *src, uint32_t span, uint32_t ip_len, uint32_t flags, uint32_t *out);

// A range registered with cgck_host_register: [lo, hi) and the device
// pointer of lo.
struct RegRange {
	uint8_t *lo, *hi;
	uint8_t *dev;
};
// Is [p, p + bytes) inside one registered range?  Fills *r when it is.
bool reg_find(const void *p, size_t bytes, RegRange *r);
// Bumped by every cgck_host_register / _unregister: a range found under one
// value stays valid while the value holds (the drop-ins' per-thread cache).
extern std::atomic<uint64_t> g_reg_gen;

// The calling thread's drop-in context (created on first use); nullptr with
// the error text set when no gfx950 device can be used.
cgck_ctx *thread_ctx();
cgck_ctx *thread_ctx_if_any(); // the context if this thread made one, else nullptr
// Report a failure of a call that has no error channel (the drop-in
// symbols): the handler of cgck_set_error_handler, then abort.
[[noreturn]] void die(const char *what);

int rss_prepare(cgck_ctx *c, const uint8_t *key, int key_size, uint32_t cnt, hipStream_t st);
int rss_note_use(cgck_ctx *c, hipStream_t st);
constexpr uint32_t kRssMaxCnt = 65536;

} // namespace cgck
#pragma GCC visibility pop
