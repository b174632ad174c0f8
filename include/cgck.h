/*
 * cgck.h — C-ABI of the MI355X (gfx950) Internet-checksum engine that stands in
 * for con-gen's checksum unit (reference: kogdenko/con-gen, subr.c:119-223).
 *
 * Two layers, one shared library (libcgck.so):
 *
 *  1. Drop-in symbols.  `in_cksum` and `udp_cksum` keep the exact prototypes of
 *     subr.h:373-374 (and therefore the `ip_cksum` / `tcp_cksum` macros of
 *     subr.h:176-177 keep working unchanged).  They are synchronous: each call
 *     runs the gfx950 kernel on the calling thread's own context (stream +
 *     pinned staging) and returns the host-order u16 the call sites store
 *     verbatim into the header.  Inside a deferred TX window
 *     (cgck_tx_begin .. cgck_tx_flush) the same symbols queue the packet and
 *     return 0; the flush fills every queued field in one batched launch
 *     (the bsd_flush / toy_flush batch point).
 *
 *  2. Batched API (`cgck_*`).  Packet batches described either by a fixed
 *     stride or by 12-byte descriptors, device-resident (all pointers are
 *     device pointers) or host-resident (pinned staging, H2D + kernel + D2H).
 *     Every entry point returns 0 or a negative errno and never aborts.
 *
 * Semantics (bit-exact with the reference on the same bytes):
 *   S   = sum of the region's little-endian 16-bit words counted from the
 *         region's first byte (odd trailing byte = low byte), plus the
 *         12-byte pseudo-header for L4 (subr.c:119-125, 197-210);
 *   out = (S mod 65535 == 0) ? 0xFFFF : 0xFFFF - (S mod 65535)
 *         (reduce(), subr.c:137-156: a folded sum of 0 maps to 0xFFFF).
 *
 * No HIP or torch types appear in any signature: streams are `void *`
 * (a hipStream_t, or NULL for the context's own stream).
 */
#ifndef CGCK_H
#define CGCK_H

#include <stdint.h>
#include <stddef.h>
#include <netinet/ip.h> /* struct ip, as subr.h:29 uses it */

#ifdef __cplusplus
extern "C" {
#endif

#define CGCK_ABI_VERSION 2

/* ------------------------------------------------------------------------ */
/* 1. Drop-in symbols (subr.h:373-374; bodies subr.c:186-195, 212-223).     */
/* ------------------------------------------------------------------------ */

/* Checksum of [data, data+len).  ip_cksum(ip) == in_cksum(ip, ip->ip_hl<<2)
 * (subr.h:176).  Callers: ip_output.c:63, ip_input.c:51, ip_icmp.c:77,191,
 * gbtcp/inet.c:322, gbtcp/tcp.c:374. */
uint16_t in_cksum(void *data, int len);

/* TCP/UDP checksum: `len` bytes at ip + ip_hl*4 plus the pseudo-header
 * {ip_src, ip_dst, 0, ip_p, htons(len)}.  tcp_cksum == udp_cksum (subr.h:177).
 * Callers: tcp_output.c:417, tcp_input.c:78, tcp_subr.c:122,
 * udp_usrreq.c:89,189, gbtcp/inet.c:145, gbtcp/tcp.c:377. */
uint16_t udp_cksum(struct ip *ip, int len);

/* ------------------------------------------------------------------------ */
/* 2. Batched API.                                                           */
/* ------------------------------------------------------------------------ */

typedef struct cgck_ctx cgck_ctx_t;

/* One packet of a descriptor batch: the IPv4 header sits at
 * base + frame_off + l3_off; ip_len bytes of datagram follow it
 * (ip_hl*4 header bytes + the L4 region).  12 bytes, 4-byte aligned. */
typedef struct cgck_desc {
	uint64_t frame_off; /* byte offset of the frame from the batch base   */
	uint16_t l3_off;    /* IPv4 header offset inside the frame (14: Ethernet) */
	uint16_t ip_len;    /* datagram bytes covered (IPv4 total length)      */
} __attribute__((packed, aligned(4))) cgck_desc_t;

/* Operation flags. */
enum {
	CGCK_RAW         = 1u << 0, /* out.lo = in_cksum(ip, ip_len): whole region, no header semantics */
	CGCK_IP          = 1u << 1, /* out.lo = ip_cksum(ip) = in_cksum(ip, ip_hl<<2) */
	CGCK_L4          = 1u << 2, /* out.hi = udp_cksum(ip, ip_len - ip_hl*4) (pseudo-header) */
	CGCK_L4_NOPSEUDO = 1u << 3, /* with CGCK_L4: out.hi = in_cksum(ip+hl, ip_len-hl) (ICMP, ip_icmp.c:77,191) */
	CGCK_ZERO_FIELDS = 1u << 4, /* read the checksum fields as zero: ip+10 and the L4 field by ip_p
	                               (TCP +16, UDP +6, ICMP +2 after the header) — the "field = 0,
	                               recompute" step every call site performs */
	CGCK_STORE       = 1u << 5, /* write out.lo to ip+10 and out.hi to the L4 field (TX fill) */
	CGCK_VERIFY      = 1u << 6, /* compare with the stored fields (implies ZERO_FIELDS), verdict bits */
	CGCK_V_IP_ZERO_IS_FFFF = 1u << 7, /* bsd44 ip_input.c:46-48: a received ip_sum of 0 counts as 0xFFFF */
	CGCK_V_UDP_ZERO_SKIP   = 1u << 8, /* udp_usrreq.c:86: uh_sum == 0 means "not checksummed" */
};
#define CGCK_GEN_BOTH    (CGCK_IP | CGCK_L4)
#define CGCK_FILL_BOTH   (CGCK_IP | CGCK_L4 | CGCK_ZERO_FIELDS | CGCK_STORE)
#define CGCK_VERIFY_BSD  (CGCK_IP | CGCK_L4 | CGCK_VERIFY | CGCK_V_IP_ZERO_IS_FFFF | CGCK_V_UDP_ZERO_SKIP)
#define CGCK_VERIFY_TOY  (CGCK_IP | CGCK_L4 | CGCK_VERIFY)

/* Verdict bits (one byte per packet). */
enum {
	CGCK_BAD_IP  = 1u << 0, /* -> ips_badsum    (netstat.h:40)  */
	CGCK_BAD_L4  = 1u << 1, /* -> tcps_rcvbadsum / udps_badsum (netstat.h:103,129) */
	CGCK_BAD_LEN = 1u << 2, /* header modes only: ip_len < 20 or ip_len < ip_hl*4
	                           (ip_input.c:24-37 drops these before any checksum):
	                           out = 0, nothing stored, not counted as bad */
};

/* Error codes are negative errno values; this gives a thread-local message. */
const char *cgck_last_error(void);
int cgck_abi_version(void);

/* Contexts: one per calling thread (a HIP stream, pinned staging, scratch).
 * A context is never shared between threads without external locking. */
int cgck_ctx_create(int device, cgck_ctx_t **out);
int cgck_ctx_destroy(cgck_ctx_t *ctx);
void *cgck_ctx_stream(cgck_ctx_t *ctx);
int cgck_ctx_sync(cgck_ctx_t *ctx);
/* Pin the context's kernel family instead of the dispatcher's choice (parity
 * tests of every family, A/B runs): "auto" (the default), "group", "lpp",
 * "lpa", "slot2", "dstr", "lpd", "lpw".  A family that cannot take a batch
 * (alignment, flags, lengths) still falls back to one that can, so results
 * stay exact.  -EINVAL for an unknown name. */
int cgck_ctx_set_kernel(cgck_ctx_t *ctx, const char *family);

/* Device-resident batches.  `out` (u32 per packet: lo16 = IP/RAW result,
 * hi16 = L4 result), `verdict` (u8 per packet) and `bad` (u32[2] running
 * counters: [0] += bad IP, [1] += bad L4) are optional (NULL).  `stream`
 * NULL = the context's stream.  Asynchronous: returns after the launch. */
int cgck_strided(cgck_ctx_t *ctx, void *base, uint64_t n, uint64_t stride,
		 uint32_t l3_off, uint32_t ip_len, uint32_t flags,
		 uint32_t *out, uint8_t *verdict, uint32_t *bad, void *stream);
int cgck_desc(cgck_ctx_t *ctx, void *base, const cgck_desc_t *desc, uint64_t n,
	      uint32_t flags, uint32_t *out, uint8_t *verdict, uint32_t *bad,
	      void *stream);

/* Shape hint for descriptor batches: their typical (mean) ip_len, default
 * 1500.  Below 1 KiB the lane-per-packet kernel is used (mixed/small packets,
 * e.g. IMIX = 354), from 1 KiB the lane-group kernel.  Any length is still
 * handled correctly; the hint only picks the faster kernel. */
int cgck_set_desc_len_hint(cgck_ctx_t *ctx, uint32_t max_ip_len);

/* Layout hint for descriptor batches.  CGCK_LAYOUT_PACKED: the frames of a
 * batch lie back to back in descriptor order (a receive burst copied into
 * one buffer, the IMIX set of BASELINE configs[3]); the dispatcher then
 * streams the buffer itself (contiguous DMA through LDS) instead of gathering
 * each frame, for mixed lengths below 1 KiB.  Results are exact for any
 * layout: 64-frame steps that are not back to back are computed frame by
 * frame, only slower.  Default CGCK_LAYOUT_ANY. */
enum { CGCK_LAYOUT_ANY = 0, CGCK_LAYOUT_PACKED = 1 };
int cgck_set_desc_layout(cgck_ctx_t *ctx, uint32_t layout);

/* Host-resident batch (ring memory), synchronous.  Registered memory
 * (cgck_host_register) is read where it lies and in-place stores land there;
 * a small pageable burst (packet bytes <= 512 KiB) is copied packet by packet
 * into pinned staging that the kernel reads; a larger pageable batch goes by
 * DMA of [base, base+bytes).  Results come back to out/verdict (and, with
 * CGCK_STORE, the filled fields into `base`).  -EINVAL when a descriptor
 * reaches past `bytes`. */
int cgck_desc_host(cgck_ctx_t *ctx, void *base, size_t bytes,
		   const cgck_desc_t *desc, uint64_t n, uint32_t flags,
		   uint32_t *out, uint8_t *verdict);

/* Zero-copy ring memory: page-lock a transport's
 * buffer pool (netmap slots, XDP UMEM, DPDK mempool) so H2D copies read it
 * directly.  Thin wrappers of hipHostRegister / hipHostUnregister. */
int cgck_host_register(void *ptr, size_t bytes);
int cgck_host_unregister(void *ptr);
/* The device view of [ptr, ptr + bytes) inside a range registered with
 * cgck_host_register (for cgck_burst_request); -ENOENT otherwise. */
int cgck_host_device_ptr(const void *ptr, size_t bytes, void **dev);

/* The drop-in symbols run on a per-thread context created on first use
 * (device from $CGCK_DEVICE, default 0).  cgck_thread_ctx returns that
 * context (creating it), so a worker's batched calls (cgck_desc_host,
 * cgck_dst_cache_host, ...) share its stream and staging with the drop-ins;
 * NULL on failure (cgck_last_error says why).  A worker thread that exits
 * calls cgck_thread_release to free it. */
cgck_ctx_t *cgck_thread_ctx(void);
int cgck_thread_release(void);

/* Per-thread device binding (one host thread per device).  A
 * worker calls cgck_thread_bind(queue_id % cgck_device_count()) in its
 * thread_init (con-gen.c:1062-1100 starts one worker per RSS queue, up to
 * N_THREADS_MAX = 32, subr.h:58) before its first checksum call; its
 * drop-in context, windows and burst server then live on that device.  The
 * binding outlives cgck_thread_release.  -EINVAL: no such device; -EBUSY:
 * the thread's context already exists on another device (release it first).
 * cgck_thread_device returns the device the thread's context is (or will be)
 * on. */
int cgck_thread_bind(int device);
int cgck_thread_device(void);

/* The drop-in symbols have no error channel (their prototypes are the
 * reference's).  When one cannot produce a result (no device, a launch or
 * synchronisation failure) it calls the handler set here with what failed
 * and cgck_last_error()'s text — con-gen passes a function that ends in its
 * panic3() (subr.c:238-261), which prints the stats and exits.  If the
 * handler returns, or none is set, the library prints the message and
 * aborts.  Process-wide; NULL restores the default. */
typedef void (*cgck_error_fn)(const char *what, const char *msg, void *arg);
void cgck_set_error_handler(cgck_error_fn fn, void *arg);

/* RX window at the transport's receive burst.
 * cgck_rx_begin computes, for every frame of the burst in one launch, the
 * values the stack's own verifiers are about to ask for — ip_cksum of the
 * header with ip_sum read as zero (ip_input.c:49-51, gbtcp/inet.c:319-322)
 * and the L4 checksum with its field read as zero: tcp_cksum / udp_cksum of
 * the segment (tcp_input.c:75-78, udp_usrreq.c:86-89, gbtcp/inet.c:142-145)
 * or, for ICMP, in_cksum of the message (ip_icmp.c:187-189).  Until
 * cgck_rx_end, this thread's drop-in in_cksum / udp_cksum calls on those
 * headers and segments (same pointer, same length) return the precomputed
 * value without touching the GPU; any other call is computed synchronously
 * as outside the window.  The stack's verify, count and drop code
 * (t_*_do_incksum 0/1/2) therefore runs unchanged.
 *
 * desc[i] = {frame offset from base, l3_off (14 for Ethernet), bytes
 * received after l3_off (ip_input's `len`)}; [base, base + bytes) must hold
 * every frame and stay unchanged (apart from the checksum fields the stack
 * zeroes and rewrites) until cgck_rx_end.  The L4 value covers
 * ntohs(ip_len) - ip_hl*4 bytes when the frame holds them.  Registered
 * memory (cgck_host_register) is read in place.  Returns the number of
 * frames precomputed, or a negative errno (-EBUSY: a window is already
 * open).  cgck_rx_end returns how many calls the window answered. */
int cgck_rx_begin(void *base, size_t bytes, const cgck_desc_t *desc, uint64_t n);
int cgck_rx_end(void);

/* Pipelined RX window: bursts in flight while the stack works.  The
 * transport posts burst k as it arrives (cgck_rx_post returns at once, the
 * burst server computing it meanwhile), then opens the window over the
 * oldest posted burst — k - 1, whose values are in by then — with
 * cgck_rx_begin_posted, runs the stack over it and closes it with
 * cgck_rx_end as above.  The ring keeps a posted burst's frames unchanged
 * until its window closes (netmap's head and DPDK's mbuf free come after
 * the stack's processing: netmap.c:116-126, dpdk.c:255-263).  Up to 64
 * bursts may be posted and not yet opened (-EBUSY beyond).  One request per
 * thread is on the burst server at a time: the bursts posted while it is
 * there go out together, as one request, when it is back, so a loop that
 * posts small bursts faster than one request's round trip pays one round
 * trip per round trip, not per burst.  Without an open burst server, or
 * when a burst does not fit it, cgck_rx_post computes the burst at once.
 * cgck_rx_post returns the frames posted (-EINVAL: a descriptor reaches
 * past `bytes`); cgck_rx_begin_posted the frames the window answers for
 * (as cgck_rx_begin), -ENOENT when nothing is posted.  Posted fills
 * (cgck_tx_post) coalesce the same way, and bursts and fills waiting
 * together over the same registered range go out as one request. */
int cgck_rx_post(void *base, size_t bytes, const cgck_desc_t *desc, uint64_t n);
int cgck_rx_begin_posted(void);

/* The drain rule.  con-gen's loop calls io_rx only on POLLIN
 * (con-gen.c:508-517), so the burst posted last before a quiet spell would
 * otherwise wait for the next frame to arrive.  Every thread_process
 * iteration that posts no burst drains: while cgck_rx_pending() > 0, the
 * transport opens the oldest posted burst (cgck_rx_begin_posted, which
 * waits for its values if the GPU is not done), runs the stack over it,
 * closes it and releases its slots.  A burst therefore
 * never waits longer than one loop iteration after its post.
 * cgck_rx_pending returns the bursts posted and not yet opened (0..64);
 * cgck_rx_ready, without waiting, 1 when the oldest one's values are in
 * (opening it will not wait), 0 while the GPU still computes it, -ENOENT
 * when nothing is posted.  A transport may also drain a ready burst early,
 * in the iteration that posted it (after check_timers, con-gen.c:524). */
int cgck_rx_pending(void);
int cgck_rx_ready(void);

/* Deferred TX fill.  Between begin and flush, the
 * drop-in in_cksum/udp_cksum calls of THIS thread that target an IPv4
 * header (len == ip_hl*4), a TCP/UDP segment, or an ICMP message right
 * after a 20-byte header of protocol 1 (icmp_send, ip_icmp.c:68-80) lying
 * inside memory registered with cgck_host_register (the transport's ring or
 * mempool, whose slots stay owned by the stack until the kick) return 0 and
 * are queued; a second call for the same header or segment replaces the
 * first.  Calls on any other memory (a stack-local struct packet, pkt_body)
 * are computed synchronously, as outside the window.  The flush computes the
 * queue in one launch and writes each result into its field (ip+10; TCP +16
 * / UDP +6 / ICMP +2 after the header); it must run before the transport
 * hands the slots to the NIC.  Returns the number of fields written, or a
 * negative errno.
 *
 * The window may stay open for the whole loop iteration,
 * so the replies the stack builds while it processes a burst (tcp_respond,
 * icmp_error, echo replies) and check_timers' keepalives are queued too.
 * A call about a frame of the open RX window is never queued (it is the
 * stack verifying what it received).  A received frame must therefore be
 * processed inside an RX window whenever the TX window is open: its verify
 * calls outside one would look like a transmit call and be queued.
 * cgck_window_stats_n's counter [4] counts queued calls on a header of the
 * last closed RX window's frames, so an integration that misses that rule
 * shows up there. */
int cgck_tx_begin(void);
int cgck_tx_flush(void);

/* Pipelined TX fill: cgck_tx_post closes the window like cgck_tx_flush but
 * returns once the fill is posted (the number of fields queued); the fields
 * are final once cgck_tx_complete, which waits for the oldest posted fill,
 * returns how many it wrote (0: none posted).  The kernel returns the
 * values and the completion writes the fields from the host, so the ring
 * lines stay in the worker's caches for the stack's next writes to those
 * slots.  The transport calls
 * it before it hands those slots to the NIC — at the next loop's kick
 * (con-gen.c:493), so the GPU computes burst k while the stack builds burst
 * k + 1.  Up to 64 fills may be posted and not yet completed: one more
 * cgck_tx_post completes the oldest first (its fields are written then); if
 * that completion fails, the new window is still posted and the oldest
 * fill's error is returned (its fields stay unwritten: the transport drops
 * or recomputes those packets). */
int cgck_tx_post(void);
int cgck_tx_complete(void);

/* Without waiting: fills posted and not yet completed (cgck_tx_pending),
 * and whether the oldest one's values are in (cgck_tx_ready: 1, so
 * cgck_tx_complete will not wait; 0 while the GPU computes it; -ENOENT
 * when none is posted).  A transport that holds each fill's slots back from
 * the NIC until its completion (netmap: `head` stops at the fill's first
 * slot; DPDK: its mbufs stay out of rte_eth_tx_burst) can complete fills as
 * they come back instead of waiting at every kick. */
int cgck_tx_pending(void);
int cgck_tx_ready(void);

/* Per-thread window counters since the thread's first call:
 * [0] drop-in calls answered by an RX window, [1] calls inside an RX window
 * computed synchronously (no match), [2] calls queued by a TX window, [3]
 * calls inside a TX window computed synchronously (memory not registered). */
int cgck_window_stats(uint64_t stats[4]);
/* The same counters and more: writes min(n, 5) of them and returns how many
 * the library keeps (5).  [4]: TX-window calls queued on the IPv4 header of a
 * frame of the last closed RX window (a received frame verified outside an RX
 * window, see cgck_tx_begin; or a received frame reused for a reply). */
int cgck_window_stats_n(uint64_t *stats, int n);

/* Burst server (latency).  Keeps up to 32 workgroups
 * (one per 64 packets of max_pkts) resident on `ctx` (NULL: this thread's
 * drop-in context) that serve host-resident batches through a mailbox (a
 * doorbell in device memory the host writes through the large BAR, or
 * host-coherent memory): cgck_desc_host, the RX window, the TX window's flush (its queue
 * read in place when it lies in one registered range, as cgck_desc_host of
 * that range) and the synchronous drop-in calls then skip the kernel launch
 * and the stream synchronisation whenever a batch fits (at most max_pkts packets and max_bytes of packet bytes; a
 * batch of more than 64 packets is split over the workgroups).  Batches
 * above the caps take the launch path, whose many workgroups read host
 * memory faster for hundreds of frames of >= 576 B: max_bytes ~96 KiB routes
 * a mixed workload best.  Each server holds a hardware
 * queue of its own, so a device takes at most 12 from a process (-EBUSY
 * beyond: that context runs its requests through launches).  The server exits after idle_ms
 * without a request (0: 200 ms) and is relaunched by the next one; close
 * stops it.  cgck_ctx_destroy and cgck_thread_release close it too. */
int cgck_burst_open(cgck_ctx_t *ctx, uint32_t max_pkts, size_t max_bytes, uint32_t idle_ms);
int cgck_burst_close(cgck_ctx_t *ctx);

/* One request to ctx's open burst server (NULL: this thread's context) over
 * memory the device already sees — [dev_base, dev_base + range), e.g. the
 * device view of a ring registered elsewhere.  The host does not check the
 * descriptors: the server checks every one against `range` on the device
 * before any load or store, and a descriptor that reaches past it fails the
 * request with -EIO: the workgroup whose slice holds it reads and stores
 * nothing (the other slices of a wide request may have been served).  Every request the library posts
 * to a server for registered memory (cgck_desc_host, the RX/TX windows)
 * carries its range the same way.  -ENOSPC: no server open, or n above its
 * max_pkts.  cgck_host_register / cgck_host_unregister drain every open
 * server before the mapping changes (the next request relaunches it), so no
 * server kernel runs across a mapping change. */
int cgck_burst_request(cgck_ctx_t *ctx, const void *dev_base, uint64_t range,
		       const cgck_desc_t *desc, uint64_t n, uint32_t flags,
		       uint32_t *out, uint8_t *verdict);

/* Synthetic batches generated on the device.  Byte j of the
 * stream is byte (j & 7) of splitmix64(seed, j >> 3); each packet then gets
 * ver/ihl 0x45, tos 0, total length, ip_p = 6 and zeroed IP/TCP checksum
 * fields.  IMIX: 64/576/1500 at 7:4:1 in a fixed 12-packet cycle, packed
 * densely, with the descriptors written to `desc`. */
int cgck_synth_strided(cgck_ctx_t *ctx, void *base, uint64_t n, uint64_t stride,
		       uint32_t ip_len, uint64_t seed, void *stream);
int cgck_synth_imix(cgck_ctx_t *ctx, void *base, cgck_desc_t *desc, uint64_t n,
		    uint64_t seed, void *stream);
uint64_t cgck_imix_bytes(uint64_t n); /* bytes an n-packet IMIX batch occupies */
/* The same IMIX frames in ring slots: frame k at k * stride + l3_off (the
 * netmap layout: 2048-byte slots, IPv4 at +14), n * stride bytes of buffer. */
int cgck_synth_imix_ring(cgck_ctx_t *ctx, void *base, cgck_desc_t *desc, uint64_t n, uint64_t stride,
			 uint32_t l3_off, uint64_t seed, void *stream);

/* ------------------------------------------------------------------------ */
/* 3. Toeplitz RSS hash (subr.c:482-530, subr.h:370-371) */
/*    and the dst-cache build that calls it (con-gen.c:291-360).             */
/* ------------------------------------------------------------------------ */

/* Drop-in symbols, prototypes of subr.h:370-371.  Synchronous, on the calling
 * thread's context (like in_cksum).  toeplitz_hash: subr.c:482-502 over
 * `cnt` bytes (cnt <= 65536; reads key[0..3] and key[4..key_size-1] as the
 * reference does).  rss_hash4: subr.c:506-530, the hash of the 12 bytes
 * {faddr, laddr, fport, lport} masked to 7 bits.  Caller: con-gen.c:338. */
uint32_t toeplitz_hash(const unsigned char *data, int cnt, const unsigned char *key, int key_size);
uint32_t rss_hash4(uint32_t laddr, uint32_t faddr, uint16_t lport, uint16_t fport,
		   unsigned char *key, int key_size);

/* Batched hash, device-resident: out[k] = toeplitz_hash(data + k*stride, cnt,
 * key, key_size) & mask (mask 0x7F = rss_hash4 on {faddr, laddr, fport,
 * lport} records of 12 bytes).  `key` is host memory (the context derives
 * and caches its byte tables).  Asynchronous. */
int cgck_toeplitz(cgck_ctx_t *ctx, const void *data, uint64_t n, uint64_t stride, uint32_t cnt,
		  const unsigned char *key, int key_size, uint32_t mask, uint32_t *out, void *stream);

/* One dst-cache entry: the fields thread_init_dst_cache fills in struct
 * ip_socket (con-gen.c:344-349; subr.h:218-228).  16 bytes. */
typedef struct cgck_dst_entry {
	uint32_t laddr; /* ipso_laddr, network order */
	uint32_t faddr; /* ipso_faddr, network order */
	uint16_t lport; /* ipso_lport, network order */
	uint16_t fport; /* ipso_fport, network order */
	uint32_t hash;  /* ipso_hash = SO_HASH(faddr, lport, fport) (subr.h:179-180) */
} cgck_dst_entry_t;

/* The struct thread fields the loop reads (subr.h:274-279, 325-328). */
typedef struct cgck_dst_params {
	uint32_t laddr_min, laddr_max; /* t_ip_laddr_min/max, host order */
	uint32_t faddr_min, faddr_max; /* t_ip_faddr_min/max, host order */
	uint16_t fport;                /* t_port, network order */
	uint8_t rss_queue_num;         /* t_rss_queue_num */
	uint8_t rss_queue_id;          /* t_rss_queue_id; the filter runs only when
	                                  id < 128 (RSS_QUEUE_ID_MAX) and num > 1 */
	const unsigned char *rss_key;  /* t_rss_key (host memory; unused without the filter) */
	int rss_key_size;              /* t_rss_key_size */
} cgck_dst_params_t;

/* Enumerate the candidate tuples in the reference's loop order (faddr
 * fastest, then the ephemeral lport 5000..65535, then laddr; the tuple count
 * is computed in 32-bit arithmetic as con-gen.c:314-315 does), keep those
 * whose rss_hash4 % queue_num == queue_id, and write the first `cap`
 * (t_dst_cache_size, >= 1) in order.  `*count` = entries written
 * (con-gen.c:356; the caller panics below t_concurrency, :357-358).
 * cgck_dst_cache: `out` and `count` are device memory, asynchronous.
 * cgck_dst_cache_host: host memory, synchronous. */
int cgck_dst_cache(cgck_ctx_t *ctx, const cgck_dst_params_t *prm, cgck_dst_entry_t *out, uint32_t cap,
		   uint32_t *count, void *stream);
int cgck_dst_cache_host(cgck_ctx_t *ctx, const cgck_dst_params_t *prm, cgck_dst_entry_t *out,
			uint32_t cap, uint32_t *count);

/* Plumbing for callers without their own runtime (tests, bench, C users).
 * A free while any burst server is resident is deferred until the last one
 * closes: hipFree / hipHostFree synchronise the device, which would wait for
 * the resident servers to idle out (the library's own buffers are handled
 * the same way). */
int cgck_device_count(void);
int cgck_dev_alloc(size_t bytes, void **ptr);
int cgck_dev_free(void *ptr);
int cgck_host_alloc(size_t bytes, void **ptr); /* pinned */
int cgck_host_free(void *ptr);
int cgck_memcpy(void *dst, const void *src, size_t bytes, void *stream); /* async, any direction */
int cgck_memset(void *dst, int value, size_t bytes, void *stream);

/* Name of the last checksum / hash kernel the context's dispatcher launched,
 * as rocprofv3 reports it (e.g. "cksum_kernel<16, 6, 1, false, true>");
 * "" before the first launch. */
const char *cgck_ctx_last_kernel(cgck_ctx_t *ctx);

/* HIP-event timing on a given stream (NULL = context stream). */
typedef struct cgck_event cgck_event_t;
int cgck_event_create(cgck_event_t **ev);
int cgck_event_destroy(cgck_event_t *ev);
int cgck_event_record(cgck_ctx_t *ctx, cgck_event_t *ev, void *stream);
int cgck_event_elapsed_ms(cgck_event_t *start, cgck_event_t *stop, float *ms);

/* Diagnostics: a plain coalesced streaming read of [src, src+bytes) (device
 * memory, 16-byte aligned) with minimal arithmetic — the practical HBM-read
 * ceiling the checksum kernels are compared with.  `sink` is a device u32. */
int cgck_probe_read(cgck_ctx_t *ctx, const void *src, uint64_t bytes, uint32_t *sink, void *stream);

/* Test hooks (tests/test_gpu_burst_seq.py; not for production callers).
 * cgck_test_burst_seq restarts ctx's open, idle burst server as if `seq` were
 * the last request served (the 32-bit seq wrap test); cgck_test_burst_stale
 * sets the done words of workgroups >= from half the seq space ahead (a word
 * untouched for 2^31 requests), which the next request must refresh.
 * -EINVAL: no server open, or a posted request not yet collected. */
int cgck_test_burst_seq(cgck_ctx_t *ctx, uint32_t seq);
int cgck_test_burst_stale(cgck_ctx_t *ctx, uint32_t from);

#ifdef __cplusplus
}
#endif
#endif /* CGCK_H */
