/*
 * Burst-level timing of SURVEY §8(f) ranks 1 and 2 through the C-ABI, called
 * the way con-gen's C code would call it (no Python per packet):
 *
 *   rx_verify — one cgck_desc_host() per receive burst over a netmap-like
 *               ring (2048-byte slots, IPv4 header at +14) with the BSD
 *               verify semantics (ip_input.c:45-58, tcp_input.c:75-85);
 *               verdicts and results come back to host memory.
 *   rx_window — the RX window: cgck_rx_begin() over the burst, then per
 *               packet the stack's own verify calls, in_cksum(ip, 20) and
 *               udp_cksum(ip, len - 20) with the fields zeroed and restored
 *               (gbtcp/inet.c:319-330, 142-153), answered from the window,
 *               then cgck_rx_end().
 *   tx_fill   — the deferred TX window on the registered ring: per packet
 *               the stack's own calls, udp_cksum(ip, len - 20) then
 *               in_cksum(ip, 20), queued between cgck_tx_begin() and
 *               cgck_tx_flush() (glue.c:15-41 batch point), the flush writing
 *               every field in place.
 *
 *   rx_reference_loop / tx_reference_loop — the same RX and TX loops (the
 *               field save / zero / restore and stores included) calling the
 *               reference's own in_cksum / udp_cksum (subr.c:186-223, built
 *               by oracle/build_ref.sh into oracle/_ref/libref_cksum.so) on
 *               one core: the CPU cost the windows replace, measured by the
 *               same harness.
 *   rx_window_pipelined / tx_fill_pipelined — the same with one burst in
 *               flight (cgck_rx_post + cgck_rx_begin_posted, cgck_tx_post +
 *               cgck_tx_complete): burst k is posted, then the stack works
 *               on burst k - 1; between bursts the thread spins
 *               TXBURST_STACK_US microseconds (default 50) for the rest of
 *               the stack's per-burst work, which the GPU overlaps.  The
 *               reported time is what the worker thread spends in the
 *               checksum path per burst — post, the wait for the previous
 *               burst's values, the stack's calls, end — with the wait alone
 *               beside it.
 *
 * RX is measured four ways: the launch path on pageable ring memory, the
 * ring registered (cgck_host_register: read where it lies), the resident
 * burst server (cgck_burst_open: no launch or stream sync per call), and
 * both; TX on the registered ring (the window queues only registered
 * memory); plus one synchronous drop-in in_cksum without and with the
 * server.  Prints one JSON line per (mode, packet length, burst).  Parity of
 * every path is covered by tests/; here each run also checks that the
 * verify passes flag exactly the packets it corrupted.
 *
 *   tools/txburst [seconds per cell, default 0.4]
 */
#include <dlfcn.h>
#include <libgen.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

#include "cgck.h"

#define SLOT 2048
#define L3 14

static double now(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static int cmpd(const void *a, const void *b)
{
	double x = *(const double *)a, y = *(const double *)b;
	return x < y ? -1 : x > y;
}

/* IPv4 + TCP packet of `len` bytes with pseudo-random payload, zero checksum fields */
static void make_packet(uint8_t *ip, int len, uint64_t *s)
{
	for (int i = 0; i < len; i++) {
		*s ^= *s << 13;
		*s ^= *s >> 7;
		*s ^= *s << 17;
		ip[i] = (uint8_t)*s;
	}
	ip[0] = 0x45;
	ip[1] = 0;
	ip[2] = (uint8_t)(len >> 8);
	ip[3] = (uint8_t)len;
	ip[9] = 6;
	ip[10] = ip[11] = 0;
	ip[20 + 16] = ip[20 + 17] = 0;
}

static double median(double *t, int n)
{
	qsort(t, n, sizeof(double), cmpd);
	return t[n / 2];
}

/* after median() sorted t: the p-th percentile */
static double pct(const double *t, int n, int p)
{
	return t[(long)n * p / 100 < n ? (long)n * p / 100 : n - 1];
}

int main(int argc, char **argv)
{
	const double budget = argc > 1 ? atof(argv[1]) : 0.4;
	const int bursts[] = {32, 64, 128, 256, 512, 1024, 2048};
	const int nb = (int)(sizeof(bursts) / sizeof(bursts[0]));
	/* 1500 B MTU frames, 576 B (con-gen's MTU 522 + headers, con-gen.c:741,
	 * rounded up to the IMIX class) and 64 B minimum frames */
	int lens[8] = {1500, 576, 64};
	int nl = 3;
	/* TXBURST_LENS=128,64: other frame lengths (con-gen's own frames are
	 * mostly 54-130 B), 40..1500 each */
	if (getenv("TXBURST_LENS")) {
		nl = 0;
		for (char *e = getenv("TXBURST_LENS"); *e && nl < 8;) {
			const int v = (int)strtol(e, &e, 10);
			if (v >= 40 && v <= 1500)
				lens[nl++] = v;
			while (*e == ',')
				e++;
			if (*e && (*e < '0' || *e > '9'))
				break;
		}
		if (!nl)
			return 2;
	}
	const int maxb = 2048, maxit = 100000;
	/* TXBURST_HUGE=1: the ring on transparent huge pages (2 MiB), as a DPDK
	 * mempool or a huge-page XDP UMEM would be; otherwise 4 KiB pages */
	uint8_t *ring;
	if (getenv("TXBURST_HUGE") && atoi(getenv("TXBURST_HUGE"))) {
		const size_t sz = (size_t)2 * maxb * SLOT, al = 2u << 20;
		uint8_t *m = mmap(NULL, sz + al, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
		ring = m == MAP_FAILED ? NULL : (uint8_t *)(((uintptr_t)m + al - 1) & ~(uintptr_t)(al - 1));
		if (ring)
			madvise(ring, sz, MADV_HUGEPAGE);
	} else {
		/* a mapping of its own, as a transport's pool is (cgck_host_register
		 * refuses the brk heap); two halves: bursts k and k - 1 */
		ring = mmap(NULL, (size_t)2 * maxb * SLOT, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
		if (ring == MAP_FAILED)
			ring = NULL;
	}
	const double stack_us = getenv("TXBURST_STACK_US") ? atof(getenv("TXBURST_STACK_US")) : 50.0;
	const int pretouch = getenv("TXBURST_PRETOUCH") && atoi(getenv("TXBURST_PRETOUCH"));
	cgck_desc_t *desc = malloc(sizeof(cgck_desc_t) * maxb);
	uint32_t *out = malloc(4 * maxb);
	uint8_t *ver = malloc(maxb);
	double *t = malloc(sizeof(double) * maxit);
	double *tc = malloc(sizeof(double) * maxit); /* RX window: the per-packet calls + rx_end only */
	double *tw = malloc(sizeof(double) * maxit); /* pipelined: the wait for the previous burst */
	double *tp = malloc(sizeof(double) * maxit); /* pipelined TX: cgck_tx_post */
	cgck_ctx_t *ctx;
	if (!ring || !desc || !out || !ver || !t || !tc || !tw || cgck_ctx_create(0, &ctx)) {
		fprintf(stderr, "txburst: setup failed: %s\n", cgck_last_error());
		return 1;
	}
	if (argc > 2 && !strcmp(argv[2], "dropin")) {
		/* drop-in latency alone: launch path, server of 1 and of 32
		 * workgroups, launch path again after they closed */
		memset(ring, 0, SLOT);
		uint64_t s0 = 1;
		make_packet(ring + L3, 64, &s0);
		/* (max_pkts, max_bytes) of the server; 0: the launch path */
		uint32_t caps[16] = {0, 64, 64, 2048, 2048, 0};
		size_t bytes[16] = {0, 64 << 10, 3 << 20, 64 << 10, 3 << 20, 0};
		int nm = 6;
		if (argc > 3) { /* txburst budget dropin max_pkts[:max_bytes] ... (0: launch path) */
			nm = 0;
			for (int a = 3; a < argc && nm < 16; a++, nm++) {
				char *colon;
				caps[nm] = (uint32_t)strtoul(argv[a], &colon, 0);
				bytes[nm] = *colon == ':' ? (size_t)strtoull(colon + 1, NULL, 0) : (size_t)caps[nm] * 1536;
			}
		}
		for (int m = 0; m < nm; m++) {
			if (caps[m] && cgck_burst_open(NULL, caps[m], bytes[m], 0)) {
				fprintf(stderr, "txburst: burst_open failed: %s\n", cgck_last_error());
				return 1;
			}
			int it = 0;
			double t0 = now();
			while (it < maxit && now() - t0 < budget) {
				double a = now();
				volatile uint16_t v = in_cksum(ring + L3, 20);
				(void)v;
				t[it++] = now() - a;
			}
			printf("{\"mode\": \"in_cksum\", \"max_pkts\": %u, \"max_bytes\": %zu, \"iters\": %d, "
			       "\"us_median\": %.2f}\n", caps[m], bytes[m], it, median(t, it) * 1e6);
			fflush(stdout);
			if (caps[m])
				cgck_burst_close(NULL);
		}
		return 0;
	}
	/* the reference's checksum unit, for the same-harness CPU rows */
	typedef uint16_t (*in_fn)(void *, int);
	typedef uint16_t (*udp_fn)(struct ip *, int);
	in_fn ref_in = NULL;
	udp_fn ref_udp = NULL;
	{
		char exe[4096];
		const ssize_t k = readlink("/proc/self/exe", exe, sizeof(exe) - 64);
		if (k > 0) {
			exe[k] = 0;
			char path[4200];
			snprintf(path, sizeof(path), "%s/../oracle/_ref/libref_cksum.so", dirname(exe));
			void *h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
			if (h) {
				ref_in = (in_fn)dlsym(h, "in_cksum");
				ref_udp = (udp_fn)dlsym(h, "udp_cksum");
			}
		}
	}
	for (int li = 0; li < nl; li++) {
		const int len = lens[li];
		uint64_t s = 0x9E3779B97F4A7C15ull;
		for (int i = 0; i < maxb; i++) {
			make_packet(ring + (size_t)i * SLOT + L3, len, &s);
			desc[i].frame_off = (uint64_t)i * SLOT;
			desc[i].l3_off = L3;
			desc[i].ip_len = (uint16_t)len;
		}
		/* fill both fields in place (the TX result a receiver would see) */
		if (cgck_desc_host(ctx, ring, (size_t)maxb * SLOT, desc, maxb,
				   CGCK_IP | CGCK_L4 | CGCK_ZERO_FIELDS | CGCK_STORE, out, NULL)) {
			fprintf(stderr, "txburst: fill failed: %s\n", cgck_last_error());
			return 1;
		}
		/* the second half (the pipelined modes' other burst): the same frames */
		memcpy(ring + (size_t)maxb * SLOT, ring, (size_t)maxb * SLOT);
		/* corrupt one payload byte of every 64th packet (both halves) */
		for (int i = 0; i < 2 * maxb; i += 64)
			ring[(size_t)i * SLOT + L3 + len - 1] ^= 0x5A;
		/* the ring as received: the reference rows and the TX rows rewrite
		 * fields, so it is put back before each RX pass */
		uint8_t *keep = malloc((size_t)2 * maxb * SLOT);
		if (!keep) {
			fprintf(stderr, "txburst: out of memory\n");
			return 1;
		}
		memcpy(keep, ring, (size_t)2 * maxb * SLOT);
		for (int bi = 0; bi < nb && ref_in && ref_udp; bi++) { /* the reference loop, same harness */
			const int R = bursts[bi];
			for (int mode = 0; mode < 2; mode++) {
				int it = 0, w = 0;
				volatile int sink = 0;
				double t0 = now();
				while (it < maxit && now() - t0 < budget) {
					double a = now();
					int bad = 0;
					for (int i = 0; i < R; i++) {
						uint8_t *ip = ring + (size_t)i * SLOT + L3;
						uint16_t saved, v;
						if (mode == 0) { /* RX: verify, field zeroed and restored */
							memcpy(&saved, ip + 10, 2);
							ip[10] = ip[11] = 0;
							v = ref_in(ip, 20);
							bad += v != saved;
							memcpy(ip + 10, &saved, 2);
							memcpy(&saved, ip + 20 + 16, 2);
							ip[20 + 16] = ip[20 + 17] = 0;
							v = ref_udp((struct ip *)ip, len - 20);
							bad += v != saved;
							memcpy(ip + 20 + 16, &saved, 2);
						} else { /* TX: fill */
							ip[20 + 16] = ip[20 + 17] = 0;
							v = ref_udp((struct ip *)ip, len - 20);
							memcpy(ip + 20 + 16, &v, 2);
							ip[10] = ip[11] = 0;
							v = ref_in(ip, 20);
							memcpy(ip + 10, &v, 2);
						}
					}
					sink += bad;
					if (w++ >= 20)
						t[it++] = now() - a;
				}
				printf("{\"mode\": \"%s\", \"pkt_len\": %d, \"burst\": %d, \"iters\": %d, \"us_median\": %.2f}\n",
				       mode ? "tx_reference_loop" : "rx_reference_loop", len, R, it, median(t, it) * 1e6);
				fflush(stdout);
			}
		}
		if (keep) {
			memcpy(ring, keep, (size_t)2 * maxb * SLOT);
		}
		/* passes: 0 launch path, 1 registered ring, 2 burst server, 3 server + registered */
		for (int pass = 0; pass < 4; pass++) {
			const int reg = pass & 1, srv = pass >= 2;
			static const char *rx_name[4] = {"rx_verify", "rx_verify_registered", "rx_verify_server",
							 "rx_verify_registered_server"};
			static const char *win_name[4] = {"rx_window", "rx_window_registered", "rx_window_server",
							  "rx_window_registered_server"};
			if (pass == 2) /* pass 1's TX cells refilled the fields: toggle the corruption back */
				for (int i = 0; i < 2 * maxb; i += 64)
					ring[(size_t)i * SLOT + L3 + len - 1] ^= 0x5A;
			if (reg && cgck_host_register(ring, (size_t)2 * maxb * SLOT)) {
				fprintf(stderr, "txburst: register failed: %s\n", cgck_last_error());
				return 1;
			}
			if (srv && (cgck_burst_open(ctx, maxb, (size_t)maxb * 1536, 0) ||
				    cgck_burst_open(NULL, maxb, (size_t)maxb * 1536, 0))) {
				fprintf(stderr, "txburst: burst_open failed: %s\n", cgck_last_error());
				return 1;
			}
			for (int bi = 0; bi < nb; bi++) {
				const int R = bursts[bi];
				const uint32_t vf = CGCK_IP | CGCK_L4 | CGCK_VERIFY | CGCK_V_IP_ZERO_IS_FFFF |
						    CGCK_V_UDP_ZERO_SKIP;
				int it = 0, bad_l4 = 0, bad_ip = 0;
				double t0 = now();
				for (int w = 0; w < 20; w++)
					cgck_desc_host(ctx, ring, (size_t)R * SLOT, desc, R, vf, out, ver);
				while (it < maxit && now() - t0 < budget) {
					double a = now();
					if (cgck_desc_host(ctx, ring, (size_t)R * SLOT, desc, R, vf, out, ver)) {
						fprintf(stderr, "txburst: verify failed: %s\n", cgck_last_error());
						return 1;
					}
					t[it++] = now() - a;
				}
				for (int i = 0; i < R; i++) {
					bad_ip += (ver[i] & CGCK_BAD_IP) != 0;
					bad_l4 += (ver[i] & CGCK_BAD_L4) != 0;
				}
				const double us = median(t, it) * 1e6;
				printf("{\"mode\": \"%s\", \"pkt_len\": %d, \"burst\": %d, \"iters\": %d, "
				       "\"us_median\": %.2f, \"mpkt_s\": %.3f, \"bad_ip\": %d, \"bad_l4\": %d, "
				       "\"bad_l4_expected\": %d}\n",
				       rx_name[pass], len, R, it, us, R / us, bad_ip, bad_l4, (R + 63) / 64);
				fflush(stdout);
			}
			for (int bi = 0; bi < nb; bi++) {
				const int R = bursts[bi];
				int it = 0, w = 0, bad_ip = 0, bad_l4 = 0;
				double t0 = now();
				while (it < maxit && now() - t0 < budget + 0.05) {
					double a = now();
					int bi_ = 0, bl_ = 0;
					if (cgck_rx_begin(ring, (size_t)R * SLOT, desc, R) != R) {
						fprintf(stderr, "txburst: rx_begin failed: %s\n", cgck_last_error());
						return 1;
					}
					const double a1 = now();
					for (int i = 0; i < R; i++) {
						uint8_t *ip = ring + (size_t)i * SLOT + L3;
						uint16_t saved, v;
						memcpy(&saved, ip + 10, 2); /* inet.c:319-330 */
						ip[10] = ip[11] = 0;
						v = in_cksum(ip, 20);
						bi_ += v != saved;
						memcpy(ip + 10, &saved, 2);
						memcpy(&saved, ip + 20 + 16, 2); /* inet.c:142-153 */
						ip[20 + 16] = ip[20 + 17] = 0;
						v = udp_cksum((struct ip *)ip, len - 20);
						bl_ += v != saved;
						memcpy(ip + 20 + 16, &saved, 2);
					}
					if (cgck_rx_end() != 2 * R) {
						fprintf(stderr, "txburst: the window answered fewer than %d calls\n", 2 * R);
						return 1;
					}
					bad_ip = bi_;
					bad_l4 = bl_;
					if (w++ >= 20) {
						tc[it] = now() - a1;
						t[it++] = now() - a;
					}
				}
				const double us = median(t, it) * 1e6, us_calls = median(tc, it) * 1e6;
				printf("{\"mode\": \"%s\", \"pkt_len\": %d, \"burst\": %d, \"iters\": %d, "
				       "\"us_median\": %.2f, \"us_calls\": %.2f, \"mpkt_s\": %.3f, \"bad_ip\": %d, "
				       "\"bad_l4\": %d, \"bad_l4_expected\": %d}\n",
				       win_name[pass], len, R, it, us, us_calls, R / us, bad_ip, bad_l4, (R + 63) / 64);
				fflush(stdout);
			}
			for (int bi = 0; bi < nb && (pass == 1 || pass == 3); bi++) { /* TX: registered ring, launch / server */
				const int R = bursts[bi];
				int it = 0, w = 0;
				double t0 = now();
				while (it < maxit && now() - t0 < budget + 0.05) {
					double a = now();
					cgck_tx_begin();
					for (int i = 0; i < R; i++) {
						uint8_t *ip = ring + (size_t)i * SLOT + L3;
						uint16_t v;
						ip[20 + 16] = ip[20 + 17] = 0; /* tcp_template: th_sum = 0 */
						v = udp_cksum((struct ip *)ip, len - 20); /* th->th_sum = tcp_cksum(...) */
						memcpy(ip + 20 + 16, &v, 2);
						ip[10] = ip[11] = 0;           /* ip->ip_sum = 0 */
						v = in_cksum(ip, 20);          /* ip->ip_sum = ip_cksum(ip) */
						memcpy(ip + 10, &v, 2);
					}
					const double a1 = now();
					const int r = cgck_tx_flush();
					if (r != 2 * R) {
						fprintf(stderr, "txburst: flush wrote %d of %d: %s\n", r, 2 * R,
							cgck_last_error());
						return 1;
					}
					if (w++ >= 20) {
						tc[it] = now() - a1;
						t[it++] = now() - a;
					}
				}
				const double us = median(t, it) * 1e6, us_flush = median(tc, it) * 1e6;
				printf("{\"mode\": \"%s\", \"pkt_len\": %d, \"burst\": %d, \"iters\": %d, "
				       "\"us_median\": %.2f, \"us_flush\": %.2f, \"mpkt_s\": %.3f}\n",
				       pass == 3 ? "tx_fill_registered_server" : "tx_fill_registered", len, R, it, us, us_flush,
				       R / us);
				fflush(stdout);
			}
			for (int bi = 0; bi < nb && pass == 3; bi++) { /* RX, one burst in flight */
				const int R = bursts[bi];
				memcpy(ring, keep, (size_t)2 * maxb * SLOT); /* both halves as received */
				int it = 0, k = 0, bad_l4 = 0, bad_ip = 0;
				double t0 = now();
				while (it < maxit && now() - t0 < budget + 0.05) {
					uint8_t *half = ring + (size_t)(k & 1) * maxb * SLOT;   /* burst k */
					uint8_t *prev = ring + (size_t)((k + 1) & 1) * maxb * SLOT; /* burst k - 1 */
					double a = now(), aw = a;
					if (cgck_rx_post(half, (size_t)R * SLOT, desc, R) != R) {
						fprintf(stderr, "txburst: rx_post failed: %s\n", cgck_last_error());
						return 1;
					}
					if (k > 0) {
						aw = now();
						if (k > 20)
							tc[it] = aw - a; /* the post */
						if (cgck_rx_begin_posted() != R) {
							fprintf(stderr, "txburst: rx_begin_posted failed: %s\n", cgck_last_error());
							return 1;
						}
						const double w = now() - aw;
						int bi_ = 0, bl_ = 0;
						for (int i = 0; i < R; i++) {
							uint8_t *ip = prev + (size_t)i * SLOT + L3;
							uint16_t saved, v;
							memcpy(&saved, ip + 10, 2);
							ip[10] = ip[11] = 0;
							v = in_cksum(ip, 20);
							bi_ += v != saved;
							memcpy(ip + 10, &saved, 2);
							memcpy(&saved, ip + 20 + 16, 2);
							ip[20 + 16] = ip[20 + 17] = 0;
							v = udp_cksum((struct ip *)ip, len - 20);
							bl_ += v != saved;
							memcpy(ip + 20 + 16, &saved, 2);
						}
						if (cgck_rx_end() != 2 * R) {
							fprintf(stderr, "txburst: the pipelined window answered fewer than %d calls\n", 2 * R);
							return 1;
						}
						bad_ip = bi_;
						bad_l4 = bl_;
						if (k > 20) {
							t[it] = now() - a;
							tw[it++] = w;
						}
					}
					k++;
					for (double s0 = now(); now() - s0 < stack_us * 1e-6;) /* the rest of the stack's work */
						;
				}
				/* drain the last posted burst */
				cgck_rx_begin_posted();
				cgck_rx_end();
				const double us = median(t, it) * 1e6, us_wait = median(tw, it) * 1e6,
					     us_post = median(tc, it) * 1e6;
				printf("{\"mode\": \"rx_window_pipelined_registered_server\", \"pkt_len\": %d, \"burst\": %d, "
				       "\"iters\": %d, \"us_median\": %.2f, \"us_wait\": %.2f, \"us_post\": %.2f, "
				       "\"stack_us\": %.1f, \"bad_ip\": %d, \"bad_l4\": %d, \"bad_l4_expected\": %d, "
				       "\"exact\": %s}\n",
				       len, R, it, us, us_wait, us_post, stack_us, bad_ip, bad_l4, (R + 63) / 64,
				       bad_ip == 0 && bad_l4 == (R + 63) / 64 ? "true" : "false");
				fflush(stdout);
			}
			for (int bi = 0; bi < nb && pass == 3; bi++) { /* TX, one fill in flight */
				const int R = bursts[bi];
				int it = 0, k = 0;
				double t0 = now();
				while (it < maxit && now() - t0 < budget + 0.05) {
					uint8_t *half = ring + (size_t)(k & 1) * maxb * SLOT;
					if (pretouch) /* lab split: the frames' lines owned by this core before the clock starts */
						for (int i = 0; i < R; i++) {
							volatile uint8_t *ip = half + (size_t)i * SLOT + L3;
							ip[36] = ip[36];
						}
					double a = now();
					cgck_tx_begin();
					for (int i = 0; i < R; i++) {
						uint8_t *ip = half + (size_t)i * SLOT + L3;
						uint16_t v;
						ip[20 + 16] = ip[20 + 17] = 0;
						v = udp_cksum((struct ip *)ip, len - 20);
						memcpy(ip + 20 + 16, &v, 2);
						ip[10] = ip[11] = 0;
						v = in_cksum(ip, 20);
						memcpy(ip + 10, &v, 2);
					}
					const double ap = now();
					if (k > 20)
						tc[it] = ap - a;
					if (cgck_tx_post() != 2 * R) {
						fprintf(stderr, "txburst: tx_post failed: %s\n", cgck_last_error());
						return 1;
					}
					double aw = now(), w = 0;
					if (k > 0) {
						if (k > 20)
							tp[it] = aw - ap;
						const int r = cgck_tx_complete(); /* burst k - 1, before its kick */
						w = now() - aw;
						if (r != 2 * R) {
							fprintf(stderr, "txburst: tx_complete wrote %d of %d: %s\n", r, 2 * R,
								cgck_last_error());
							return 1;
						}
						if (k > 20) {
							t[it] = now() - a;
							tw[it++] = w;
						}
					}
					k++;
					for (double s0 = now(); now() - s0 < stack_us * 1e-6;)
						;
				}
				cgck_tx_complete();
				const double us = median(t, it) * 1e6, us_wait = median(tw, it) * 1e6;
				const double p10 = pct(t, it, 10) * 1e6, p90 = pct(t, it, 90) * 1e6;
				const double us_calls = median(tc, it) * 1e6, calls_p90 = pct(tc, it, 90) * 1e6;
				const double us_post = median(tp, it) * 1e6, post_p90 = pct(tp, it, 90) * 1e6;
				printf("{\"mode\": \"tx_fill_pipelined_registered_server\", \"pkt_len\": %d, \"burst\": %d, "
				       "\"iters\": %d, \"us_median\": %.2f, \"us_p10\": %.2f, \"us_p90\": %.2f, "
				       "\"us_wait\": %.2f, \"us_calls\": %.2f, \"us_calls_p90\": %.2f, \"us_post\": %.2f, "
				       "\"us_post_p90\": %.2f, \"stack_us\": %.1f}\n",
				       len, R, it, us, p10, p90, us_wait, us_calls, calls_p90, us_post, post_p90, stack_us);
				fflush(stdout);
			}
			if (srv) {
				cgck_burst_close(ctx);
				cgck_burst_close(NULL);
			}
			if (reg)
				cgck_host_unregister(ring);
		}
		free(keep);
		/* drop-in latency: one synchronous in_cksum(ip, 20), launch path vs server */
		for (int srv = 0; srv < 2; srv++) {
			int it = 0;
			if (srv && cgck_burst_open(NULL, 64, 1 << 16, 0)) {
				fprintf(stderr, "txburst: burst_open failed: %s\n", cgck_last_error());
				return 1;
			}
			double t0 = now();
			while (it < maxit && now() - t0 < budget) {
				double a = now();
				volatile uint16_t v = in_cksum(ring + L3, 20);
				(void)v;
				t[it++] = now() - a;
			}
			printf("{\"mode\": \"%s\", \"pkt_len\": 20, \"burst\": 1, \"iters\": %d, "
			       "\"us_median\": %.2f}\n", srv ? "in_cksum_server" : "in_cksum", it, median(t, it) * 1e6);
			fflush(stdout);
			if (srv)
				cgck_burst_close(NULL);
		}
	}
	cgck_ctx_destroy(ctx);
	cgck_thread_release();
	return 0;
}
