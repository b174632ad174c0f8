// cgck_internal.h — shared between the kernels and the host C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/cgck.h"

// Run-time A/B knobs ($CGCK_KERNEL, $CGCK_LPW_WPC, ...) exist only in the lab
// build (libcgck_lab.so, -DCGCK_LAB): there CGCK_ENV reads the environment;
// in the product library it is a null pointer, so every knob takes its
// measured default and its name is not even in the binary.  $CGCK_DEVICE
// (the drop-in symbols' device) is the product's one environment variable.
#if CGCK_LAB
#include <stdlib.h>
#define CGCK_ENV(name) getenv(name)
#else
#define CGCK_ENV(name) ((const char *)nullptr)
#endif

namespace cgck {

// Internal flag (never part of the public enum): skip the BAD_LEN rule so the
// drop-in udp_cksum keeps the pure-function semantics of subr.c:212-223 even
// for malformed headers.
constexpr uint32_t kFlagNoLenCheck = 1u << 15;
// Internal flag of the RX window (cgck_rx_begin): the L4 result of each
// packet follows its own protocol, as the stack's verifiers do — ICMP (ip_p 1)
// is in_cksum(ip + hl, len - hl) with its field at +2 (ip_icmp.c:187-189),
// everything else udp_cksum with the pseudo-header (tcp_input.c:75-78,
// udp_usrreq.c:86-89).  Group kernel only.
constexpr uint32_t kFlagL4Auto = 1u << 14;
// Internal flag of the RX window: descriptor ip_len is the bytes the frame
// holds after l3_off (ip_input's `len`); the group kernel itself decides, as
// cgck_rx_begin's host walk used to, which calls the stack can make on the
// frame (ip_input.c:28-44, 76; tcp_input.c:67; udp_usrreq.c:65;
// ip_icmp.c:177; gbtcp/inet.c:282-314) and covers min(ntohs(ip_len), len)
// bytes.  Per frame it writes KParams.meta: kRxOkIp | kRxOkL4 | kRxIcmp,
// ip_hl * 4 in bits 8-15, ntohs(ip_len) - ip_hl * 4 in bits 16-31.
constexpr uint32_t kFlagRx = 1u << 13;
constexpr uint32_t kRxOkIp = 1, kRxOkL4 = 2, kRxIcmp = 4;
// Internal flag: a host-resident region bound by PCIe round trips (the
// drop-in symbols' one region): take the group kernel, whose one block reads
// the region at once, whatever the lane kernels' preconditions say (lpd for
// a 20-byte in_cksum read its DMA steps over the fabric: 31 vs 14 us).
constexpr uint32_t kFlagGroup = 1u << 12;

// The flag sets of the windows' requests (cgck_dropin.cpp): every frame of a
// receive burst (its meta word, both results by ip_p, fields read as zero),
// and a transmit fill's headers and segments (both fields read as zero;
// kFlagL4Auto too when the fill holds ICMP messages).  The burst server's
// one-workgroup body is compiled for each (burst_body_spec, cgck_group.hip).
constexpr uint32_t kRxFlags = CGCK_IP | CGCK_L4 | CGCK_ZERO_FIELDS | kFlagL4Auto | kFlagRx;
constexpr uint32_t kTxFlags = CGCK_IP | CGCK_L4 | CGCK_ZERO_FIELDS;

constexpr uint32_t kImixCycleBytes = 4252; // 7*64 + 4*576 + 1500

// Zeroed device bytes per context: 64 lines of 64 B, so dummy loads can be
// spread over L2 channels instead of all hitting one line.
constexpr uint32_t kZeroBytes = 64 * 64;

struct KParams {
	const uint8_t *base;
	const cgck_desc_t *desc; // nullptr: strided batch
	uint64_t n;
	uint64_t stride;
	uint32_t l3_off;
	uint32_t ip_len;
	uint32_t flags;
	uint32_t *out;
	uint8_t *verdict;
	uint32_t *bad;
	uint32_t contig; // set by the launcher: contiguous block ranges
	const void *zero; // kZeroBytes zero bytes of device memory (safe target for clamped loads)
	uint32_t *meta;   // kFlagRx only: one word per packet (see kFlagRx)
};

// Mailbox of the burst server (cgck_group.hip), in host-coherent pinned
// memory.  Two request slots, so one request can be in flight while the host
// posts the next (the pipelined RX / TX windows): request seq lives in slot
// seq & 1 — its block at bstage + (seq & 1) * cap, its outputs at bresp +
// (seq & 1) * burst_resp_slot(max_pkts), its mailbox word req[seq & 1] =
// seq | n << 32, stored (release) after the block.  Seqs run 1, 2, ... by
// burst_next (never 0, parity alternating through the wrap), and the server
// serves them strictly in that order: its leader workgroup polls the slot of
// the seq after the last it served and relays each request to the others
// through device memory, so each learns the packet count, and with it its
// share, from its poll.  Workgroup j of the W = burst_wgs(n, K) that serve a
// request answers with done[j] = seq (release) once its outputs are visible;
// a workgroup that refuses its slice (burst_hdr_ok / desc_inside) first
// stores refused[seq & 1] = seq.
constexpr uint32_t kBurstMaxWG = 32; // workgroups of a server (K)
constexpr uint32_t kBurstOneWG = 64; // packets one workgroup serves alone (one wide read of the block)
constexpr uint32_t kBurstPerWG = 64; // packets per workgroup of a wider request (default)
struct BurstBox {
	uint64_t req[2];     // host -> device: seq | n << 32 of the request in slot seq & 1
	uint32_t stop;       // host -> device: exit now
	uint32_t bad_req;    // device -> host: slices refused by the server's checks (a count)
	uint64_t idle_ticks; // 100 MHz ticks without a request before the server exits
	uint32_t refused[2]; // device -> host: seq of the last refused request in each slot
	uint64_t lab_cyc;    // lab build: workgroup 0's shader clocks (s_memtime) over the compute phase
	uint64_t lab_body;   // lab build: thread 0's shader clocks over the one-workgroup body call alone
	uint32_t pad[2];
	uint32_t done[kBurstMaxWG]; // device -> host: the last request workgroup j served
	uint8_t alive[kBurstMaxWG]; // host sets 1 at launch; workgroup j clears its byte on exit
	uint64_t lab_t[4];   // lab build: workgroup 0's s_memrealtime at seen / read / computed / published
};
static_assert(sizeof(BurstBox) == 64 + 5 * kBurstMaxWG + 32, "mailbox line, the done lines, the alive lines, lab");

// The seq after s: 1, 2, ..., 0xfffffffe, 1, ...: never 0 (the relay's
// "nothing posted"), and s & 1 alternates through the wrap.
__host__ __device__ constexpr uint32_t burst_next(uint32_t s) { return s >= 0xfffffffeu ? 1u : s + 1u; }

// Workgroups that serve a request of n packets on a server of K with `per`
// packets per workgroup: one up to kBurstOneWG packets (it reads the whole
// small block in one round trip), then one per `per` packets, at most K.
// A wide request's packet reads over the fabric are bound by the device's
// aggregate host-read rate, not by one CU: 2048 x 64 B in place took 25.3 /
// 31.2 / 44.4 / 43.9 us at 64 / 32 / 16 / 8 packets per workgroup
// (tools/srvlat, profiles/r03/burst/srvlat_per_wg.log), so 64 it is.
__host__ __device__ constexpr uint32_t burst_wgs(uint32_t n, uint32_t K, uint32_t per)
{
	return n <= kBurstOneWG ? 1u : ((n + per - 1) / per < K ? (n + per - 1) / per : K);
}

// Header of a request block (the first 64 bytes of the burst staging), then
// the n descriptors at d_off = 64, then (base == 0) the packet bytes.  A
// request served by one workgroup is copied into device scratch with one wide
// read of the block's first kBurstFirst bytes — every thread's loads in
// flight together, one host round trip for a small request's header,
// descriptors and packet bytes — and the rest of a larger block in a second
// pass.  Workgroup j of a wider request reads the header and its own slice of
// the descriptors in one round trip and the packet bytes where they lie.
struct BurstReq {
	uint32_t n;       // packets
	uint32_t flags;   // CGCK_* flags
	uint32_t max_len; // longest ip_len (picks the lane shape)
	uint32_t bytes;   // size of the request block, this header included
	uint64_t base;    // device view of packets read in place (registered memory); 0: in the block
	uint32_t d_off;   // descriptors: offset in the block
	uint32_t p_off;   // packet bytes (base == 0): offset in the block
	uint64_t range;   // base != 0: bytes readable from base; the server refuses a descriptor past it
	uint32_t n1;      // 0 < n1 < n: descriptors [n1, n) take flags2 (a receive burst and a TX
	uint32_t flags2;  // fill sharing one request); 0: every descriptor takes flags
	uint32_t pad[4];
};
static_assert(sizeof(BurstReq) == 64, "one header line");
constexpr uint32_t kBurstFirst = 8192;

// Outputs of a server request of n packets, host-coherent and packed by n
// (not by the server's capacity), so a small request's outputs share one
// page: [out u32 x n | meta u32 x n | verdict u8 x n], each part 64-byte
// aligned.  (With the verdicts at a capacity-sized offset, 16 KiB away, a
// one-packet request took 36.8 us instead of 9.5: tools/txburst dropin.)
__host__ __device__ constexpr uint32_t burst_meta_off(uint32_t n) { return (4 * n + 63) & ~63u; }
__host__ __device__ constexpr uint32_t burst_ver_off(uint32_t n) { return 2 * burst_meta_off(n); }
// Bytes of one slot's outputs for requests of up to max_pkts packets.
__host__ __device__ constexpr uint32_t burst_resp_slot(uint32_t max_pkts)
{
	return (burst_ver_off(max_pkts) + max_pkts + 63) & ~63u;
}
// req: slot 0's block (slot 1's at req + cap); resp: slot 0's outputs (slot
// 1's at resp + burst_resp_slot(max_pkts)); dcmd: 24 bytes of uncached device
// memory, the leader's relay words (one per slot, then the exit word), zeroed
// here on the launch stream before the launch; start_seq: the last request
// completed (the server serves burst_next(start_seq) first); epoch: nonzero,
// new for every launch; opts: lab A/B bits (0 in the product).
// door: the two mailbox words the leader polls (box->req in host memory, or
// the device-memory doorbell the host writes through the large BAR); stopw:
// the stop word it polls with them (box->stop, or beside the doorbell); vblk:
// the device-memory request slots of small blocks (kBurstFirst bytes each,
// nullptr: none), used by a request whose mailbox word has kBurstVram set in
// its count.
hipError_t launch_burst_server(BurstBox *box, const uint64_t *door, const uint32_t *stopw, const uint8_t *req,
			       const uint8_t *vblk, uint8_t *scratch, uint8_t *resp, uint64_t *dcmd, const void *zero,
			       uint32_t cap, uint32_t max_pkts, uint32_t wgs, uint32_t per_wg, uint32_t start_seq,
			       uint32_t epoch, uint32_t opts, hipStream_t st);
// In the mailbox word's count (bits 32-63): the request's block is in the
// device-memory slot (vblk) of its parity, not in the host staging.
constexpr uint32_t kBurstVram = 1u << 31;

// Kernel selection flags (see cgck_dispatch.cpp) and the measured defaults
// (tools/sweep.py; profiles/r01).  The group kernel streams whole lines per
// wave-instruction, so nontemporal loads + contiguous block ranges win
// (1500 B: 5.79 -> 6.18 TB/s); the lane kernels re-touch each line from
// several instructions, so they want cached loads (NT: -30..-50 %).
constexpr int kNT = 16, kContig = 32, kExplicit = 64;
constexpr int kPacked = 128; // the context's descriptor layout hint is CGCK_LAYOUT_PACKED
constexpr uint32_t kGroupFromLen = 1024; // typical length from which the group kernel is used
constexpr uint32_t kLppUpToLen = 128;    // lane-per-packet up to here, lane-per-slot above
constexpr uint32_t kLpwFromLen = 256;    // back-to-back frames from here stream through LDS (lpw)
constexpr int kDefaultLppShape = 2;       // see launch_lpp (6 chunks up front, predicated: best on 64 B)
constexpr bool kDefaultGroupNT = true, kDefaultGroupContig = true;
constexpr bool kDefaultLaneNT = false, kDefaultLaneContig = false;
// Dense strided batches of >= 1 KiB frames take dstr_kernel (cgck_dense.hip,
// LDS-DMA steps of 4 frames with a writer wave): 80.3-82.0 % vs the group
// kernel's 78.6-81.5 % in the same process (tools/dstr_sweep.sh,
// profiles/r02/dense/).  The first LDS-DMA stream kernel (cgck_stream.hip,
// 76.9 % vs 77.9 %) stays in the lab build.
// Batched Toeplitz hash over dense 12-byte tuples: 0 two-group loop, 2 A/B
// pipelined (cgck_rss.hip).
constexpr int kDefaultRssVariant = 2;

// Toeplitz RSS hash (cgck_rss.hip; subr.c:482-530).  `tab` = cnt x 256 u32
// byte tables derived from the key on the host (rss_tables in cgck_api.cpp).
constexpr uint32_t kRssLdsMaxCnt = 36; // tables up to 36 KiB are staged in LDS

struct RssParams {
	const uint8_t *data;
	uint64_t n;
	uint64_t stride;
	uint32_t cnt;
	uint32_t mask;
	const uint32_t *tab;
	uint32_t *out;
};

// dst-cache build (cgck_rss.hip; con-gen.c:291-360).
struct DstParams {
	uint32_t laddr_min, faddr_min;
	uint32_t nf;             // faddr count (t_ip_faddr_max - t_ip_faddr_min + 1), nonzero
	uint32_t n;              // tuple count, u32 as con-gen.c:314-315 computes it
	uint32_t q64, r64;       // 64 / nf, 64 % nf
	uint32_t fport_be;       // t_port as stored (network order)
	uint32_t hconst;         // the fport bytes' share of the hash
	uint32_t filter;         // RSS filter on (con-gen.c:337)
	uint32_t cap;            // t_dst_cache_size (> 0)
	uint32_t ntiles;         // ceil(n / (256 * iters))
	uint32_t iters;          // per-wave iterations of 64 tuples per tile (dst_iters)
	uint64_t pass_lo, pass_hi; // bit h set: (h % t_rss_queue_num) == t_rss_queue_id, h in 0..127
	const uint32_t *tab;     // 12 x 256 byte tables of the key
	void *out;               // cgck_dst_entry_t[cap]
	uint32_t *ctl;           // [0] ticket, [1] done, [2] timeout; zeroed per launch
	uint32_t *count;         // entries written (con-gen.c:356); set by the kernel when n > 0
	uint64_t *status;        // one look-back word per tile; zeroed per launch
};

hipError_t launch_toeplitz(const RssParams &p, int num_cus, hipStream_t st);
hipError_t launch_dst_cache(const DstParams &p, int num_cus, hipStream_t st);
uint32_t dst_iters(uint32_t n, uint32_t cap, bool filter, uint64_t pass_lo, uint64_t pass_hi, int num_cus);

hipError_t launch_cksum(const KParams &p, uint32_t len_hint, int num_cus, int kernel, hipStream_t st);

// The kernel a launcher just launched, by the name rocprofv3 reports (without
// namespace and argument list); cgck_ctx_last_kernel reads it back.  Each
// launch site interns its name once (CGCK_NOTE_KERNEL) and stores the pointer.
extern thread_local const char *t_kernel;
const char *intern(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
#define CGCK_NOTE_KERNEL(...)                                                   \
	do {                                                                    \
		static const char *const note_ = ::cgck::intern(__VA_ARGS__);    \
		::cgck::t_kernel = note_;                                       \
	} while (0)
constexpr const char *tf(bool b) { return b ? "true" : "false"; }
hipError_t launch_synth_fill(uint8_t *base, uint64_t nbytes, uint64_t seed, int num_cus, hipStream_t st);
hipError_t launch_synth_stamp(uint8_t *base, uint64_t n, uint64_t stride, uint32_t len, int num_cus,
			      hipStream_t st);
hipError_t launch_probe_read(const void *src, uint64_t bytes, uint32_t *sink, int num_cus, int variant,
			     hipStream_t st);
hipError_t launch_synth_imix(uint8_t *base, uint32_t *desc, uint64_t n, int num_cus, hipStream_t st);
hipError_t launch_synth_ring(uint8_t *base, uint32_t *desc, uint64_t n, uint64_t stride, uint32_t l3_off, int num_cus,
			     hipStream_t st);

} // namespace cgck
