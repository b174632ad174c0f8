/*
 * txloop — con-gen's worker loop at the checksum boundary, through the C-ABI
 * from C, the way thread_process (con-gen.c:484-538) would run it with both
 * windows open across the whole iteration:
 *
 *   cgck_tx_complete()                 the previous iteration's fill, before
 *   io_tx()                            the kick (con-gen.c:493)
 *   cgck_tx_begin()
 *   io_rx: cgck_rx_post(burst k)       the frames that just arrived;
 *          cgck_rx_begin_posted()      the window over burst k - 1: per frame
 *          ip_input -> tcp_input       the stack's verify calls (field saved,
 *                                      zeroed, restored) and, in the "reply"
 *                                      mix, the segment it sends back built
 *                                      in a transmit slot (tcp_respond's
 *                                      tcp_cksum + ip_output's ip_cksum,
 *                                      tcp_subr.c:93-123), queued by the TX
 *                                      window; cgck_rx_end()
 *   the rest of the stack's work       a spin of `ns` per frame (README.md:6:
 *                                      ~4 Mpps a core, ~250 ns a frame), or a
 *                                      fixed 50 us per burst
 *   bsd_flush: cgck_tx_post()
 *
 * The reference row runs the same loop with the reference's own in_cksum /
 * udp_cksum (oracle/_ref/libref_cksum.so, subr.c:186-223) called in place.
 * The synchronous row opens the RX window with cgck_rx_begin and flushes with
 * cgck_tx_flush in the same iteration.  Per (mix, budget, burst, form) one
 * JSON line: the worker thread's microseconds in the checksum path per
 * iteration (everything but the spin), the part of it spent waiting for the
 * GPU (RX window open + TX completion), and the post-to-verdict latency of a
 * burst (its post to the end of its window: one loop period, or the GPU's
 * time when that is longer).  Each run checks itself: every window flags
 * exactly the frames it corrupted, and sampled replies carry the reference's
 * checksums.
 *
 * "lone" rows: one burst posted and, nothing arriving after it, drained at
 * once by the next iteration (the drain rule, include/cgck.h): the latency
 * from its post to its window's end.
 *
 *   tools/txloop [seconds per cell, default 0.2]
 *   TXLOOP_LEN=64  TXLOOP_BURSTS=1,2,4,8,16,32,64,256,2048  TXLOOP_NS=0,250
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <errno.h>
#include <pthread.h>
#include <sched.h>
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
#define MAXB 2048
#define MAXIT 200000

typedef uint16_t (*in_fn)(void *, int);
typedef uint16_t (*udp_fn)(struct ip *, int);

static double now(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static int cmpd(const void *a, const void *b)
{
	const double x = *(const double *)a, y = *(const double *)b;
	return x < y ? -1 : x > y;
}

/* sorts t; the p-th percentile */
static double pct(double *t, int n, int p)
{
	if (n <= 0)
		return 0;
	qsort(t, n, sizeof(double), cmpd);
	return t[(long)n * p / 100 < n ? (long)n * p / 100 : n - 1];
}

/* TXLOOP_SLEEP=1: the stack's other work is slept instead of spun (the
 * workers mode's control for the host's CPU quota: 32 spinning workers on a
 * box that grants 16 CPUs are throttled whatever the GPU does) */
static int g_sleep;

static void spin(double sec)
{
	if (g_sleep && sec > 0) {
		const struct timespec ts = {0, (long)(sec * 1e9)};
		nanosleep(&ts, NULL);
		return;
	}
	for (const double s0 = now(); now() - s0 < sec;)
		;
}

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
	ip[36] = ip[37] = 0;
}

/* the stack's verify of one received TCP/IPv4 frame (ip_input.c:45-58,
 * tcp_input.c:75-85, fields restored as gbtcp/inet.c does): bad checks */
static inline int verify(uint8_t *ip, int len, in_fn fin, udp_fn fudp)
{
	uint16_t saved, v;
	int bad = 0;
	memcpy(&saved, ip + 10, 2);
	ip[10] = ip[11] = 0;
	v = fin(ip, 20);
	bad += v != saved;
	memcpy(ip + 10, &saved, 2);
	memcpy(&saved, ip + 36, 2);
	ip[36] = ip[37] = 0;
	v = fudp((struct ip *)ip, len - 20);
	bad += v != saved;
	memcpy(ip + 36, &saved, 2);
	return bad;
}

/* tcp_respond(NULL, ip, th, ...) into a transmit slot (tcp_subr.c:93-123):
 * the template from the received header, the two checksum calls */
static inline void reply(uint8_t *tx, const uint8_t *rx, in_fn fin, udp_fn fudp)
{
	uint16_t v;
	memcpy(tx, rx, 40);
	tx[2] = 0;
	tx[3] = 40;
	memcpy(tx + 12, rx + 16, 4);
	memcpy(tx + 16, rx + 12, 4);
	memcpy(tx + 20, rx + 22, 2);
	memcpy(tx + 22, rx + 20, 2);
	tx[32] = 0x50;
	tx[33] = 0x14; /* RST | ACK */
	tx[36] = tx[37] = 0;
	v = fudp((struct ip *)tx, 20);
	memcpy(tx + 36, &v, 2);
	tx[10] = tx[11] = 0;
	v = fin(tx, 20);
	memcpy(tx + 10, &v, 2);
}

struct cell {
	double *worker, *wait, *lat;
	int it, itl, bad_rx, bad_tx_checked, bad_tx;
	double total; /* worker seconds over the recorded iterations */
	long bursts;  /* bursts they processed */
	double max_iter; /* the longest iteration (all of it, spin included), warm-up too */
	int max_at;      /* at which iteration */
	int iters_all;   /* iterations run, warm-up included */
};

static in_fn ref_in;
static udp_fn ref_udp;
static double g_check; /* seconds spent checking replies (kept out of the worker's time) */

/* replies of slots [0, R) checked against the reference's values */
static int check_replies(const uint8_t *txh, int R)
{
	const double t0 = now();
	int bad = 0;
	const int idx[3] = {0, R / 2, R - 1};
	for (int j = 0; j < 3; j++) {
		uint8_t c[64];
		memcpy(c, txh + (size_t)idx[j] * SLOT + L3, 40);
		uint16_t s_ip, s_tcp, v;
		memcpy(&s_ip, c + 10, 2);
		memcpy(&s_tcp, c + 36, 2);
		c[36] = c[37] = 0;
		v = ref_udp((struct ip *)c, 20);
		bad += v != s_tcp;
		memcpy(c + 36, &v, 2);
		c[10] = c[11] = 0;
		bad += ref_in(c, 20) != s_ip;
	}
	g_check += now() - t0;
	return bad;
}

/* The full-transmit-ring regime: with no free slot, the stack builds the
 * segment in its stack-local struct packet (bsd44/tcp_output.c:60,
 * netmap.c:76-78, dpdk.c:232-236) and parks it with add_pending_packet
 * (subr.c:264-286).  That memory is not registered, so the TX window computes
 * both checksums synchronously (cgck_window_stats [3]).  Every 16th reply is
 * checked against the reference's values (time kept out of the worker's). */
static int reply_body(const uint8_t *rx, in_fn fin, udp_fn fudp, int i)
{
	uint8_t pkt_body[128];
	reply(pkt_body, rx, fin, fudp);
	if (i % 16)
		return 0;
	const double t0 = now();
	uint8_t c[64];
	memcpy(c, pkt_body, 40);
	uint16_t s_ip, s_tcp, v;
	memcpy(&s_ip, c + 10, 2);
	memcpy(&s_tcp, c + 36, 2);
	c[36] = c[37] = 0;
	v = ref_udp((struct ip *)c, 20);
	int bad = v != s_tcp;
	memcpy(c + 36, &v, 2);
	c[10] = c[11] = 0;
	bad += ref_in(c, 20) != s_ip;
	g_check += now() - t0;
	return bad;
}

/* mix 3, the full-transmit-ring regime with the integration of INTEGRATION.md
 * §2: the stack builds the segment in a pending packet taken from a
 * registered pool (not the stack-local pkt_body), so the TX window queues its
 * calls as for a ring slot; once the fill covering it has completed, the
 * transport drains it into the ring (add_pending_packet's copy, subr.c:264-
 * 286, then the ring copy when a slot frees): modelled as one 54-byte copy a
 * reply into a ring area, in the worker's time. */
static __thread int g_pend;
static __thread uint8_t g_ring[MAXB * 64];

static void drain_pending(const uint8_t *tx0, long first, long cnt)
{
	for (long i = 0; i < cnt; i++)
		memcpy(g_ring + (size_t)(i % MAXB) * 64, tx0 + (size_t)((first + i) % (2 * MAXB)) * SLOT, L3 + 40);
}

/* the coalesced form's posted fills: their first reply slot and count */
struct fills {
	long start[64], cnt[64], nrep[64];
	int h, n;
	long cursor, busy; /* next free slot; slots held by posted fills */
};

/* a fill of `nrep` replies from cursor + gap (gap: the ring's tail skipped,
 * so a fill's slots never wrap and the window keeps its address order) */
static void fill_push(struct fills *f, long gap, long nrep)
{
	const int i = (f->h + f->n) % 64;
	f->start[i] = f->cursor + gap;
	f->cnt[i] = gap + nrep;
	f->nrep[i] = nrep;
	f->n++;
	f->cursor += gap + nrep;
	f->busy += gap + nrep;
}

/* complete the oldest fill (waits if it is not back); its first reply checked */
static int fill_done(struct fills *f, int mix, const uint8_t *tx0, struct cell *c)
{
	const int done = cgck_tx_complete();
	if (done < 0)
		return done;
	const long cnt = f->cnt[f->h], nrep = f->nrep[f->h];
	if (g_pend && nrep > 0)
		drain_pending(tx0, f->start[f->h], nrep);
	if (mix && nrep > 0) {
		c->bad_tx += done != 2 * nrep;
		c->bad_tx += check_replies(tx0 + (size_t)(f->start[f->h] % (2 * MAXB)) * SLOT, 1);
		c->bad_tx_checked++;
	}
	f->busy -= cnt;
	f->h = (f->h + 1) % 64;
	f->n--;
	return 0;
}

/* One worker's ring: a pool as a netmap pool holds both rings (two receive
 * halves, bursts k and k - 1; two transmit halves, fills k and k - 1), the
 * descriptors of each receive half, and the post timestamps. */
struct wk {
	uint8_t *pool, *rxh[2], *txh[2];
	size_t pool_bytes;
	cgck_desc_t *descs[2];
	double *tpost;
	int len;
};

static int cell_alloc(struct cell *c)
{
	c->worker = malloc(sizeof(double) * MAXIT);
	c->wait = malloc(sizeof(double) * MAXIT);
	c->lat = malloc(sizeof(double) * MAXIT);
	return c->worker && c->wait && c->lat ? 0 : -1;
}

/* A worker's pool: MAXB frames of `len` bytes in each receive half, every
 * 64th corrupted, checksummed by the sender with the reference functions. */
static int wk_setup(struct wk *W, int len)
{
	const size_t half = (size_t)MAXB * SLOT;
	W->len = len;
	W->pool_bytes = 4 * half;
	W->pool = mmap(NULL, W->pool_bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
	W->tpost = malloc(sizeof(double) * (MAXIT + 64));
	W->descs[0] = malloc(sizeof(cgck_desc_t) * MAXB);
	W->descs[1] = malloc(sizeof(cgck_desc_t) * MAXB);
	if (W->pool == MAP_FAILED || !W->tpost || !W->descs[0] || !W->descs[1])
		return -1;
	W->rxh[0] = W->pool;
	W->rxh[1] = W->pool + half;
	W->txh[0] = W->pool + 2 * half;
	W->txh[1] = W->pool + 3 * half;
	uint64_t s = 0x9E3779B97F4A7C15ull;
	for (int i = 0; i < MAXB; i++) {
		uint8_t *ip = W->rxh[0] + (size_t)i * SLOT + L3;
		make_packet(ip, len, &s);
		uint16_t v = ref_udp((struct ip *)ip, len - 20); /* the sender's fill (reference functions) */
		memcpy(ip + 36, &v, 2);
		v = ref_in(ip, 20);
		memcpy(ip + 10, &v, 2);
		if (i % 64 == 0) /* every 64th frame corrupted */
			ip[len - 1] ^= 0x5A;
		/* every post names the whole pool, as a transport's does (one base,
		 * the frames by offset), so bursts posted back to back can share a
		 * request */
		W->descs[0][i].frame_off = (uint64_t)i * SLOT;
		W->descs[0][i].l3_off = L3;
		W->descs[0][i].ip_len = (uint16_t)len;
		W->descs[1][i] = W->descs[0][i];
		W->descs[1][i].frame_off += half;
	}
	memcpy(W->rxh[1], W->rxh[0], half);
	return 0;
}

/* One (form, mix, burst, stack budget) cell of con-gen's loop on this thread
 * for `budget` seconds; 0, or -1 on a library error (cgck_last_error). */
static int run_cell(struct wk *W, int form, int mix, int R, double ns, double fixed_us, double budget,
		    struct cell *cp)
{
	struct cell c = *cp;
	uint8_t *const pool = W->pool, *const *rxh = W->rxh, *const *txh = W->txh;
	const size_t pool_bytes = W->pool_bytes;
	cgck_desc_t *const *descs = W->descs;
	double *tpost = W->tpost;
	const int len = W->len;
	const double other = (R * ns + fixed_us * 1000) * 1e-9;
	const int expect = (R + 63) / 64;
	in_fn lib_in = (in_fn)in_cksum;
	udp_fn lib_udp = (udp_fn)udp_cksum;
	/* mix 2: the replies go to the stack-local struct packet (a full
	 * transmit ring), mix 1 to transmit slots; below, `mix` is the latter */
	const int body = mix == 2;
	g_pend = mix == 3; /* replies in registered pending packets, drained after their fill */
	mix = body ? 0 : g_pend ? 1 : mix;
	c.it = c.itl = c.bad_rx = c.bad_tx = c.bad_tx_checked = 0;
	c.total = 0;
	c.bursts = 0;
	c.max_iter = 0;
	c.max_at = -1;
	int k = 0;
	long copened = 0; /* coalesced form: bursts opened */
	struct fills cf;
	memset(&cf, 0, sizeof(cf));
	double ph[8] = {0};
	int nopen = 0;
	const double t0 = now();
	while (c.it < MAXIT && now() - t0 < budget) {
		const int rec = k >= 20;
		g_check = 0;
		double a = now(), w = 0, lat = 0;
		int nburst = form == 1 ? k > 0 : 1; /* bursts this iteration processed */
		int bad = 0;
		uint8_t *tx = txh[k & 1];
		if (form == 0) {
			uint8_t *rx = rxh[k & 1];
			for (int i = 0; i < R; i++) {
				uint8_t *ip = rx + (size_t)i * SLOT + L3;
				bad += verify(ip, len, ref_in, ref_udp);
				if (body)
					c.bad_tx += reply_body(ip, ref_in, ref_udp, i);
				if (mix)
					reply(tx + (size_t)i * SLOT + L3, ip, ref_in, ref_udp);
				if (g_pend)
					drain_pending(tx, i, 1);
			}
			lat = now() - a;
		} else if (form == 1) {
			double w0 = now();
			const int done = cgck_tx_complete(); /* fill k - 1 */
			w += now() - w0;
			if (done < 0)
				return -1;
			if (g_pend && k > 0 && done == 2 * R)
				drain_pending(txh[(k + 1) & 1], 0, R);
			if (mix && k > 0 && done == 2 * R) {
				c.bad_tx += check_replies(txh[(k + 1) & 1], R);
				c.bad_tx_checked++;
			}
			cgck_tx_begin();
			tpost[k] = now();
			if (cgck_rx_post(pool, pool_bytes, descs[k & 1], R) != R)
				return -1;
			if (k > 0) {
				uint8_t *rx = rxh[(k + 1) & 1];
				w0 = now();
				if (cgck_rx_begin_posted() != R)
					return -1;
				w += now() - w0;
				for (int i = 0; i < R; i++) {
					uint8_t *ip = rx + (size_t)i * SLOT + L3;
					bad += verify(ip, len, lib_in, lib_udp);
					if (body)
						c.bad_tx += reply_body(ip, lib_in, lib_udp, i);
					if (mix)
						reply(tx + (size_t)i * SLOT + L3, ip, lib_in, lib_udp);
				}
				if (cgck_rx_end() != 2 * R)
					return -1;
				lat = now() - tpost[k - 1];
			} else {
				bad = expect;
			}
		} else if (form == 3) {
			/* the kick releases the fills that are back
			 * (no wait unless 48 are outstanding); burst k
			 * is posted; every burst whose values are in
			 * is processed, oldest first (no wait unless
			 * 48 are outstanding).  Replies go to a rolling
			 * cursor over both transmit halves; a fill's
			 * slots are reused only after it completed. */
			double w0 = now();
			ph[0] = w0;
			while (cf.n > 0 && (cgck_tx_ready() == 1 || cf.n >= 48)) {
				if (fill_done(&cf, mix, txh[0], &c) < 0)
					return -1;
			}
			w += now() - w0;
			ph[1] = now();
			cgck_tx_begin();
			tpost[k % 64] = now();
			if (cgck_rx_post(pool, pool_bytes, descs[k & 1], R) != R)
				return -1;
			ph[2] = now();
			nopen = 0;
			int got = 0;
			long cur = 0; /* this iteration's reply slots */
			const long at = cf.cursor % (2 * MAXB);
			const long gap = mix && at + R > 2 * MAXB ? 2 * MAXB - at : 0;
			const long room = 2 * MAXB - (at + gap) % (2 * MAXB);
			for (;;) {
				const int pend = cgck_rx_pending();
				const int rdy = pend ? cgck_rx_ready() : 0;
				if (!pend || (rdy != 1 && pend < 48) || (mix && cur + R > room))
					break;
				w0 = now();
				while (cf.n > 0 && cf.busy + gap + cur + R > 2 * MAXB)
					if (fill_done(&cf, mix, txh[0], &c) < 0)
						return -1;
				if (cgck_rx_begin_posted() != R)
					return -1;
				w += now() - w0;
				if (nopen < 4)
					ph[3 + nopen++] = now() - w0;
				uint8_t *rx = rxh[copened & 1];
				for (int i = 0; i < R; i++) {
					uint8_t *ip = rx + (size_t)i * SLOT + L3;
					bad += verify(ip, len, lib_in, lib_udp);
					if (body)
						c.bad_tx += reply_body(ip, lib_in, lib_udp, i);
					if (mix)
						reply(txh[0] + (size_t)((cf.cursor + gap + cur + i) % (2 * MAXB)) *
								       SLOT +
							      L3,
						      ip, lib_in, lib_udp);
				}
				if (mix)
					cur += R;
				if (cgck_rx_end() != 2 * R)
					return -1;
				lat += now() - tpost[copened % 64];
				copened++;
				got++;
			}
			bad = got ? (bad == got * expect ? expect : -1) : expect;
			lat = got ? lat / got : 0;
			nburst = got;
			fill_push(&cf, cur ? gap : 0, cur);
		} else {
			uint8_t *rx = rxh[k & 1];
			cgck_tx_begin();
			double w0 = now();
			if (cgck_rx_begin(pool, pool_bytes, descs[k & 1], R) != R)
				return -1;
			w += now() - w0;
			for (int i = 0; i < R; i++) {
				uint8_t *ip = rx + (size_t)i * SLOT + L3;
				bad += verify(ip, len, lib_in, lib_udp);
				if (body)
					c.bad_tx += reply_body(ip, lib_in, lib_udp, i);
				if (mix)
					reply(tx + (size_t)i * SLOT + L3, ip, lib_in, lib_udp);
			}
			if (cgck_rx_end() != 2 * R)
				return -1;
			lat = now() - a;
		}
		const double a_spin = now();
		spin(other);
		const double spun = now() - a_spin;
		if (form == 1 || form == 3) {
			const double tp0 = now();
			if (cgck_tx_post() < 0)
				return -1;
			if (form == 3 && now() - a > 0.02) /* a slow iteration: where its time went */
				fprintf(stderr,
					"txloop: slow iteration %d (%.1f ms): fills %.3f, rx_post %.3f, opens %d (%.3f %.3f %.3f "
					"%.3f), tx_post %.3f ms; fills out %d\n",
					k, (now() - a) * 1e3, (ph[1] - ph[0]) * 1e3, (ph[2] - ph[1]) * 1e3, nopen, ph[3] * 1e3,
					ph[4] * 1e3, ph[5] * 1e3, ph[6] * 1e3, (now() - tp0) * 1e3, cf.n);
		} else if (form == 2) {
			const double w0 = now();
			if (cgck_tx_flush() != (mix ? 2 * R : 0))
				return -1;
			if (g_pend)
				drain_pending(tx, 0, R);
			w += now() - w0;
			if (mix) {
				c.bad_tx += check_replies(tx, R);
				c.bad_tx_checked++;
			}
		}
		c.bad_rx += bad != expect;
		if (now() - a > c.max_iter) {
			c.max_iter = now() - a;
			c.max_at = k;
		}
		if (rec) {
			c.total += now() - a - spun - g_check;
			c.bursts += nburst;
			c.worker[c.it] = now() - a - spun - g_check;
			c.wait[c.it] = w;
			c.it++;
			if (lat > 0) /* (the coalesced form: iterations that opened bursts) */
				c.lat[c.itl++] = lat;
		}
		k++;
	}
	if (form == 1 || form == 3) { /* drain: the bursts and fills left */
		while (cgck_rx_pending() > 0 && cgck_rx_begin_posted() >= 0)
			cgck_rx_end();
		while (cgck_tx_pending() > 0)
			cgck_tx_complete();
		memset(&cf, 0, sizeof(cf));
	}
	c.iters_all = k;
	*cp = c;
	return 0;
}

/* ------------------------------------------------------------------------
 * N workers (TXLOOP_WORKERS=1,8,16,32): con-gen's normal mode, one worker
 * thread per RSS queue (con-gen.c:1062-1100, up to N_THREADS_MAX 32,
 * subr.h:58), each pinned to its own CPU, with its own pool, its own drop-in
 * context bound to device queue % devices (cgck_thread_bind) and its own
 * burst server, all running the same cell at once.  Per N and form one JSON
 * line: the per-thread us per burst (median / p90 / max over the threads),
 * the threads' p90 iteration, latency, and whether every thread stayed exact.
 * The reference form runs the same threads without the GPU: its slowdown
 * with N is the host's own (cores, caches, the CPU quota), the control for
 * the GPU forms'.
 *   TXLOOP_MW_BURST (64)  TXLOOP_MW_NS (250)  TXLOOP_MW_MIX (1: with replies)
 * ---------------------------------------------------------------------- */
#define MW_MAXT 64
#define MW_FORMS 3

struct mw {
	int id, cpu, nforms;
	int forms[MW_FORMS];
	int R, mix;
	double ns, budget;
	struct wk W;
	struct cell c;
	int rc, dev, server;
	char err[200];
	/* per form: us per burst, p50 / p90 iteration, p50 latency, bursts, exact */
	double per[MW_FORMS], w50[MW_FORMS], w90[MW_FORMS], l50[MW_FORMS];
	long bursts[MW_FORMS];
	int exact[MW_FORMS];
};

static pthread_barrier_t g_bar;

static void mw_fail(struct mw *m, const char *what)
{
	if (!m->rc) {
		m->rc = -1;
		snprintf(m->err, sizeof(m->err), "%s: %s", what, cgck_last_error());
	}
}

static void *mw_thread(void *arg)
{
	struct mw *m = arg;
	cpu_set_t cs;
	CPU_ZERO(&cs);
	CPU_SET(m->cpu, &cs);
	pthread_setaffinity_np(pthread_self(), sizeof(cs), &cs);
	const int nd = cgck_device_count();
	if (nd < 1 || cgck_thread_bind(m->id % nd) != 0)
		mw_fail(m, "cgck_thread_bind");
	m->dev = cgck_thread_device();
	if (!m->rc && cgck_host_register(m->W.pool, m->W.pool_bytes) != 0)
		mw_fail(m, "cgck_host_register");
	pthread_barrier_wait(&g_bar); /* every ring registered (each registration stops every server) */
	/* a device takes up to 16 resident servers from a process (-EBUSY
	 * beyond): such a worker runs without one (its requests launch) */
	m->server = 0;
	if (!m->rc) {
		const int rc = cgck_burst_open(NULL, MAXB, (size_t)MAXB * 1536, 0);
		if (rc == 0)
			m->server = 1;
		else if (rc != -EBUSY)
			mw_fail(m, "cgck_burst_open");
	}
	pthread_barrier_wait(&g_bar);
	for (int f = 0; f < m->nforms; f++) {
		const int form = m->forms[f];
		if (!m->rc && form != 0) /* warm the server and the queues, not recorded */
			if (run_cell(&m->W, form, m->mix, m->R, m->ns, 0, 0.02, &m->c) < 0)
				mw_fail(m, "warm-up");
		pthread_barrier_wait(&g_bar); /* every thread runs the same cell at once */
		if (!m->rc && run_cell(&m->W, form, m->mix, m->R, m->ns, 0, m->budget, &m->c) < 0)
			mw_fail(m, "cell");
		struct cell *c = &m->c;
		m->bursts[f] = c->bursts;
		m->per[f] = c->bursts ? c->total / c->bursts * 1e6 : -1;
		m->w50[f] = c->it ? pct(c->worker, c->it, 50) * 1e6 : -1;
		m->w90[f] = c->it ? pct(c->worker, c->it, 90) * 1e6 : -1;
		m->l50[f] = c->itl ? pct(c->lat, c->itl, 50) * 1e6 : -1;
		m->exact[f] = !m->rc && c->bursts > 0 && c->bad_rx == 0 && c->bad_tx == 0;
		pthread_barrier_wait(&g_bar);
	}
	cgck_burst_close(NULL);
	pthread_barrier_wait(&g_bar); /* every server closed before the mappings change */
	cgck_host_unregister(m->W.pool);
	cgck_thread_release();
	return NULL;
}

static int cmpd_desc_free(const void *a, const void *b) { return cmpd(a, b); }

/* median / p90 / max / min of the threads' values (v is sorted) */
static void mw_stats(double *v, int n, double out[4])
{
	qsort(v, n, sizeof(double), cmpd_desc_free);
	out[0] = v[n / 2];
	out[1] = v[(long)n * 90 / 100 < n ? (long)n * 90 / 100 : n - 1];
	out[2] = v[n - 1];
	out[3] = v[0];
}

static int multi_main(double budget, int len)
{
	int counts[8], nc = 0;
	for (char *e = getenv("TXLOOP_WORKERS"); *e && nc < 8;) {
		const int v = (int)strtol(e, &e, 10);
		if (v >= 1 && v <= MW_MAXT)
			counts[nc++] = v;
		while (*e == ',')
			e++;
	}
	const int R = getenv("TXLOOP_MW_BURST") ? atoi(getenv("TXLOOP_MW_BURST")) : 64;
	const double ns = getenv("TXLOOP_MW_NS") ? atof(getenv("TXLOOP_MW_NS")) : 250;
	const int mix = getenv("TXLOOP_MW_MIX") ? atoi(getenv("TXLOOP_MW_MIX")) : 1;
	g_sleep = getenv("TXLOOP_SLEEP") && atoi(getenv("TXLOOP_SLEEP"));
	if (R < 1 || R > MAXB / 2)
		return 2;
	static const char *fname[4] = {"reference", "pipelined", "sync", "coalesced"};
	const int forms[MW_FORMS] = {0, 3, 1};
	cpu_set_t all;
	int cpus[1024], ncpu = 0;
	if (sched_getaffinity(0, sizeof(all), &all) == 0)
		for (int i = 0; i < CPU_SETSIZE && ncpu < 1024; i++)
			if (CPU_ISSET(i, &all))
				cpus[ncpu++] = i;
	if (ncpu == 0)
		return 1;
	char quota[64] = "unknown";
	FILE *fq = fopen("/sys/fs/cgroup/cpu.max", "r");
	if (fq) {
		if (fgets(quota, sizeof(quota), fq))
			quota[strcspn(quota, "\n")] = 0;
		fclose(fq);
	}
	static struct mw M[MW_MAXT];
	int maxn = 0;
	for (int i = 0; i < nc; i++)
		maxn = counts[i] > maxn ? counts[i] : maxn;
	for (int t = 0; t < maxn; t++) /* pools made once; each run registers them anew */
		if (wk_setup(&M[t].W, len) != 0 || cell_alloc(&M[t].c) != 0) {
			fprintf(stderr, "txloop: out of memory\n");
			return 1;
		}
	for (int ci = 0; ci < nc; ci++) {
		const int N = counts[ci];
		pthread_t th[MW_MAXT];
		pthread_barrier_init(&g_bar, NULL, N);
		for (int t = 0; t < N; t++) {
			struct mw *m = &M[t];
			m->id = t;
			m->cpu = cpus[(ncpu / 2 + t) % ncpu]; /* from the middle of the set, as bench.py pins one */
			m->nforms = MW_FORMS;
			memcpy(m->forms, forms, sizeof(forms));
			m->R = R;
			m->mix = mix;
			m->ns = ns;
			m->budget = budget;
			m->rc = 0;
			m->err[0] = 0;
			pthread_create(&th[t], NULL, mw_thread, m);
		}
		for (int t = 0; t < N; t++)
			pthread_join(th[t], NULL);
		pthread_barrier_destroy(&g_bar);
		for (int f = 0; f < MW_FORMS; f++) {
			double per[MW_MAXT], w90[MW_MAXT], l50[MW_MAXT], sp[4], s90[4], sl[4];
			int exact = 1, np = 0, nl = 0;
			long bursts = 0;
			for (int t = 0; t < N; t++) {
				exact = exact && M[t].exact[f];
				bursts += M[t].bursts[f];
				if (M[t].per[f] >= 0) {
					per[np] = M[t].per[f];
					w90[np++] = M[t].w90[f];
				}
				if (M[t].l50[f] >= 0)
					l50[nl++] = M[t].l50[f];
			}
			printf("{\"mode\": \"workers\", \"workers\": %d, \"form\": \"%s\", \"mix\": \"%s\", \"pkt_len\": %d, "
			       "\"burst\": %d, \"stack_ns_per_frame\": %.0f, \"stack_work\": \"%s\", \"cpus\": %d, \"cpu_max\": \"%s\", "
			       "\"bursts\": %ld",
			       N, fname[forms[f]], mix ? "rx+reply" : "rx", len, R, ns, g_sleep ? "slept" : "spun", ncpu, quota,
			       bursts);
			if (np) {
				mw_stats(per, np, sp);
				mw_stats(w90, np, s90);
				printf(", \"us_per_burst\": {\"median\": %.3f, \"p90\": %.3f, \"max\": %.3f, \"min\": %.3f}"
				       ", \"us_iter_p90\": {\"median\": %.3f, \"max\": %.3f}",
				       sp[0], sp[1], sp[2], sp[3], s90[0], s90[2]);
			} else {
				printf(", \"us_per_burst\": null");
			}
			if (nl) {
				mw_stats(l50, nl, sl);
				printf(", \"us_latency\": {\"median\": %.3f, \"max\": %.3f}", sl[0], sl[2]);
			}
			printf(", \"per_thread_us\": [");
			for (int t = 0; t < N; t++)
				printf("%s%.3f", t ? ", " : "", M[t].per[f]);
			printf("], \"devices\": [");
			for (int t = 0; t < N; t++)
				printf("%s%d", t ? ", " : "", M[t].dev);
			int nsrv = 0;
			for (int t = 0; t < N; t++)
				nsrv += M[t].server;
			printf("], \"servers\": %d, \"exact\": %s", nsrv, exact ? "true" : "false");
			for (int t = 0; t < N; t++)
				if (M[t].rc) {
					printf(", \"error\": \"thread %d: %s\"", t, M[t].err);
					break;
				}
			printf("}\n");
			fflush(stdout);
		}
	}
	return 0;
}

int main(int argc, char **argv)
{
	const double budget = argc > 1 ? atof(argv[1]) : 0.2;
	const int len = getenv("TXLOOP_LEN") ? atoi(getenv("TXLOOP_LEN")) : 64;
	int bursts[16] = {1, 2, 4, 8, 16, 32, 64, 256, 2048}, nb = 9;
	double nsl[8] = {0, 250};
	int nns = 2;
	if (getenv("TXLOOP_BURSTS")) {
		nb = 0;
		for (char *e = getenv("TXLOOP_BURSTS"); *e && nb < 16;) {
			const int v = (int)strtol(e, &e, 10);
			if (v >= 1 && v <= MAXB)
				bursts[nb++] = v;
			while (*e == ',')
				e++;
		}
	}
	if (getenv("TXLOOP_NS")) {
		nns = 0;
		for (char *e = getenv("TXLOOP_NS"); *e && nns < 7;) {
			nsl[nns++] = strtod(e, &e);
			while (*e == ',')
				e++;
		}
	}
	if (len < 40 || len > 1500)
		return 2;
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
	if (!ref_in || !ref_udp) {
		fprintf(stderr, "txloop: oracle/_ref/libref_cksum.so not found (make -C oracle ref)\n");
		return 1;
	}
	if (getenv("TXLOOP_WORKERS"))
		return multi_main(budget, len);
	struct wk W0;
	struct cell c;
	if (wk_setup(&W0, len) != 0 || cell_alloc(&c) != 0) {
		fprintf(stderr, "txloop: out of memory\n");
		return 1;
	}
	uint8_t *pool = W0.pool, **rxh = W0.rxh, **txh = W0.txh;
	const size_t pool_bytes = W0.pool_bytes;
	cgck_desc_t **descs = W0.descs;
	if (cgck_host_register(pool, pool_bytes) || cgck_burst_open(NULL, MAXB, (size_t)MAXB * 1536, 0)) {
		fprintf(stderr, "txloop: setup failed: %s\n", cgck_last_error());
		return 1;
	}
	in_fn lib_in = (in_fn)in_cksum;
	udp_fn lib_udp = (udp_fn)udp_cksum;
	/* where a small burst's fixed cost goes: the coalesced loop at one frame
	 * a burst and 250 ns of stack work a frame, each call timed (mean ns) */
	if (getenv("TXLOOP_SPLIT")) {
		/* TXLOOP_SPLIT_R: frames a burst (1), TXLOOP_SPLIT_NS: stack ns a frame (250) */
		const int R = getenv("TXLOOP_SPLIT_R") ? atoi(getenv("TXLOOP_SPLIT_R")) : 1,
			  split_reply = atoi(getenv("TXLOOP_SPLIT")) == 2;
		const double sns = getenv("TXLOOP_SPLIT_NS") ? atof(getenv("TXLOOP_SPLIT_NS")) : 250;
		if (R < 1 || R > MAXB / 2)
			return 2;
		double acc[10] = {0}, slow_t = 0;
		long slow_n = 0, forced = 0, maxpend = 0;
		long cnt[10] = {0}, k = 0, opened = 0;
		static const char *nm[10] = {"tx_ready+complete", "tx_begin", "rx_post", "rx_pending+ready",
					     "rx_begin_posted", "verify (+reply) calls", "rx_end", "tx_post", "spin", "iteration"};
		/* the lab library's phase totals inside the Poster, when loaded */
		void (*lab_times)(double *) = (void (*)(double *))dlsym(RTLD_DEFAULT, "cgck_lab_post_times");
		double lt[16] = {0};
		const double t0 = now();
		if (lab_times)
			lab_times(lt);
		while (now() - t0 < budget * 4) {
			double a = now(), b;
			const double it0 = a;
			while (cgck_tx_pending() > 0 && cgck_tx_ready() == 1)
				cgck_tx_complete();
			b = now(); acc[0] += b - a; cnt[0]++; a = b;
			cgck_tx_begin();
			b = now(); acc[1] += b - a; cnt[1]++; a = b;
			cgck_rx_post(pool, pool_bytes, descs[k & 1], R);
			b = now(); acc[2] += b - a; cnt[2]++; a = b;
			for (;;) {
				const int pend = cgck_rx_pending();
				const int rdy = pend ? cgck_rx_ready() : 0;
				b = now(); acc[3] += b - a; cnt[3]++; a = b;
				if (!pend || (rdy != 1 && pend < 48))
					break;
				forced += rdy != 1;
				maxpend = pend > maxpend ? pend : maxpend;
				cgck_rx_begin_posted();
				b = now(); acc[4] += b - a; cnt[4]++;
				if (b - a > 1e-6) { /* the opens that waited (or collected) */
					slow_n++;
					slow_t += b - a;
				}
				a = b;
				for (int i = 0; i < R; i++) {
					uint8_t *ip = rxh[opened & 1] + (size_t)i * SLOT + L3;
					verify(ip, len, lib_in, lib_udp);
					if (split_reply) /* the fill's slots: one transmit half a fill */
						reply(txh[k & 1] + (size_t)i * SLOT + L3, ip, lib_in, lib_udp);
				}
				b = now(); acc[5] += b - a; cnt[5]++; a = b;
				cgck_rx_end();
				b = now(); acc[6] += b - a; cnt[6]++; a = b;
				opened++;
			}
			cgck_tx_post();
			b = now(); acc[7] += b - a; cnt[7]++; a = b;
			spin(R * sns * 1e-9);
			b = now(); acc[8] += b - a; cnt[8]++;
			acc[9] += b - it0;
			cnt[9]++;
			k++;
		}
		while (cgck_rx_pending() > 0 && cgck_rx_begin_posted() >= 0)
			cgck_rx_end();
		while (cgck_tx_pending() > 0)
			cgck_tx_complete();
		/* lab: one host load of a mailbox / done / alive word while the server polls */
		int (*box_probe)(void *, int, double *) = (int (*)(void *, int, double *))dlsym(RTLD_DEFAULT, "cgck_lab_box_probe");
		double bp[4] = {0};
		if (box_probe)
			box_probe(NULL, 2000, bp);
		printf("{\"box_load_ns\": {\"mailbox\": %.1f, \"refused\": %.1f, \"done\": %.1f, \"alive\": %.1f}}\n", bp[0],
		       bp[1], bp[2], bp[3]);
		printf("{\"mode\": \"split\", \"reply\": %d, \"burst\": %d, \"stack_ns_per_frame\": %.0f, "
		       "\"iterations\": %ld, \"bursts_opened\": %ld",
		       split_reply, R, sns, k, opened);
		for (int i = 0; i < 10; i++)
			printf(", \"%s_ns\": %.1f", nm[i], cnt[i] ? acc[i] / cnt[i] * 1e9 : 0.0);
		printf(", \"opens_over_1us\": %ld, \"their_mean_us\": %.2f, \"opens_not_ready\": %ld, \"max_pending\": %ld",
		       slow_n, slow_n ? slow_t / slow_n * 1e6 : 0.0, forced, maxpend);
		if (lab_times) { /* per iteration: ns in each phase (TSC ticks, scaled), and its calls */
			static const char *ph[7] = {"lab_ready", "lab_collect", "lab_copy_out", "lab_send",
						    "lab_wait_lock", "lab_wait_loop", "spare"};
			const double tk0 = (double)__builtin_ia32_rdtsc(), c0 = now();
			spin(0.02);
			const double ns_per_tick = (now() - c0) * 1e9 / ((double)__builtin_ia32_rdtsc() - tk0);
			lab_times(lt);
			for (int i = 0; i < 6; i++)
				printf(", \"%s_ns_per_it\": %.1f, \"%s_calls_per_it\": %.3f, \"%s_ns_per_call\": %.1f", ph[i],
				       lt[2 * i] * ns_per_tick / k, ph[i], lt[2 * i + 1] / k, ph[i],
				       lt[2 * i + 1] ? lt[2 * i] * ns_per_tick / lt[2 * i + 1] : 0.0);
		}
		printf("}\n");
		return 0;
	}
	static const char *forms[4] = {"reference", "pipelined", "sync", "coalesced"};
	/* TXLOOP_MIXES: 0 rx, 1 rx + replies in transmit slots, 2 rx + replies
	 * in the stack-local packet (a full transmit ring), 3 the same regime
	 * with the pending packets in a registered pool (drained into the ring
	 * after their fill completes); default 0,1 */
	int mixes[4] = {0, 1, 2, 3}, nmix = 2;
	if (getenv("TXLOOP_MIXES")) {
		nmix = 0;
		for (char *e = getenv("TXLOOP_MIXES"); *e && nmix < 4;) {
			const int v = (int)strtol(e, &e, 10);
			if (v >= 0 && v <= 3)
				mixes[nmix++] = v;
			while (*e == ',')
				e++;
		}
	}
	/* TXLOOP_FORMS (0 reference, 1 pipelined, 2 sync, 3 coalesced; default all)
	 * and TXLOOP_REPEAT (each cell that many times): a repro harness */
	int formlist[4] = {0, 1, 2, 3}, nforms = 4;
	if (getenv("TXLOOP_FORMS")) {
		nforms = 0;
		for (char *e = getenv("TXLOOP_FORMS"); *e && nforms < 4;) {
			const int v = (int)strtol(e, &e, 10);
			if (v >= 0 && v <= 3)
				formlist[nforms++] = v;
			while (*e == ',')
				e++;
		}
	}
	const int nrep = getenv("TXLOOP_REPEAT") && atoi(getenv("TXLOOP_REPEAT")) > 0 ? atoi(getenv("TXLOOP_REPEAT")) : 1;
	static const char *mixname[4] = {"rx", "rx+reply", "rx+reply(full ring)", "rx+reply(full ring, registered pending)"};
	for (int mi = 0; mi < nmix; mi++) {
		const int mix = mixes[mi];
		for (int bud = 0; bud <= nns; bud++) {
			const double ns = bud < nns ? nsl[bud] : 0, fixed_us = bud < nns ? 0 : 50;
			for (int bi = 0; bi < nb; bi++) {
				const int R = bursts[bi];
				/* the full-ring mix pays two synchronous requests a reply
				 * (~12 us): 2048 frames take ~25 ms an iteration, too long
				 * for a cell's budget and its 20 unrecorded iterations */
				if (mix == 2 && R > 256)
					continue;
				for (int fi = 0; fi < nforms * nrep; fi++) {
					const int form = formlist[fi % nforms];
					if (run_cell(&W0, form, mix, R, ns, fixed_us, budget, &c) < 0)
						goto fail;
					const int n = c.it;
					const double wm = pct(c.worker, n, 50) * 1e6, w90 = pct(c.worker, n, 90) * 1e6;
					const double wt = pct(c.wait, n, 50) * 1e6;
					const double lm = pct(c.lat, c.itl, 50) * 1e6, l90 = pct(c.lat, c.itl, 90) * 1e6;
					/* A cell that recorded no burst measured nothing: its
					 * figures are null and it is not exact (bench.py then
					 * never counts it as beating the reference). */
					char per[32], wk[96], lt[64];
					const int none = c.bursts == 0;
					snprintf(per, sizeof(per), none ? "null" : "%.3f", none ? 0.0 : c.total / c.bursts * 1e6);
					snprintf(wk, sizeof(wk), n ? "%.3f, \"us_worker_p90\": %.3f, \"us_wait\": %.3f"
								   : "null, \"us_worker_p90\": null, \"us_wait\": null",
						 wm, w90, wt);
					snprintf(lt, sizeof(lt), c.itl ? "%.3f, \"us_latency_p90\": %.3f" : "null, \"us_latency_p90\": null",
						 lm, l90);
					printf("{\"mode\": \"loop\", \"form\": \"%s\", \"mix\": \"%s\", \"pkt_len\": %d, "
					       "\"burst\": %d, \"stack_ns_per_frame\": %.0f, \"stack_us_fixed\": %.0f, "
					       "\"iters\": %d, \"iters_all\": %d, \"bursts\": %ld, \"max_iter_us\": %.1f, \"max_iter_at\": %d, "
					       "\"us_per_burst\": %s, \"us_worker\": %s, \"us_latency\": %s, \"exact\": %s}\n",
					       forms[form], mixname[mix], len, R, ns, fixed_us, n, c.iters_all, c.bursts,
					       c.max_iter * 1e6, c.max_at, per, wk, lt,
					       !none && c.bad_rx == 0 && c.bad_tx == 0 ? "true" : "false");
					fflush(stdout);
				}
			}
		}
	}
	/* the drain rule alone: one burst, nothing after it */
	for (int bi = 0; bi < nb; bi++) {
		const int R = bursts[bi];
		int n = 0, bad = 0;
		const double t0 = now();
		while (n < MAXIT && now() - t0 < budget) {
			const double a = now();
			if (cgck_rx_post(pool, pool_bytes, descs[0], R) != R || cgck_rx_pending() != 1)
				goto fail;
			if (cgck_rx_begin_posted() != R) /* the next iteration: nothing arrived, drain */
				goto fail;
			int b = 0;
			for (int i = 0; i < R; i++)
				b += verify(rxh[0] + (size_t)i * SLOT + L3, len, lib_in, lib_udp);
			if (cgck_rx_end() != 2 * R)
				goto fail;
			bad += b != (R + 63) / 64;
			c.lat[n++] = now() - a;
			spin(20e-6); /* a quiet spell */
		}
		const double lm = pct(c.lat, n, 50) * 1e6, l90 = pct(c.lat, n, 90) * 1e6;
		printf("{\"mode\": \"lone\", \"pkt_len\": %d, \"burst\": %d, \"iters\": %d, \"us_latency\": %.3f, "
		       "\"us_latency_p90\": %.3f, \"exact\": %s}\n",
		       len, R, n, lm, l90, bad == 0 ? "true" : "false");
		fflush(stdout);
	}
	cgck_burst_close(NULL);
	cgck_host_unregister(pool);
	cgck_thread_release();
	return 0;
fail:
	fprintf(stderr, "txloop: %s\n", cgck_last_error());
	return 1;
}
