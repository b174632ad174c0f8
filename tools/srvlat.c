/* Burst-server latency breakdown (lab build, libcgck_lab.so): one
 * cgck_desc_host verify request at a time on a registered ring of 2048 B
 * slots (IPv4 at +14), with workgroup 0's device timestamps
 * (cgck_lab_burst_times: seen, block read, computed, published; 100 MHz)
 * against the host's post and done times.  Prints, per burst size, the
 * median of each phase in microseconds.  `srvlat LEN raw` sends CGCK_RAW
 * requests instead of the BSD verify flags.  Not product code. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/mman.h>
#include <string.h>
#include <time.h>

#include "cgck.h"

int cgck_lab_burst_times(cgck_ctx_t *c, uint64_t dev[5], uint64_t host[2]);
uint64_t cgck_lab_burst_body(cgck_ctx_t *c);

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

static double med(double *v, int n)
{
	qsort(v, n, sizeof(double), cmpd);
	return v[n / 2];
}

int main(int argc, char **argv)
{
	const int len = argc > 1 ? atoi(argv[1]) : 64;
	const int maxb = 2048, it = 2000;
	/* a mapping of its own (cgck_host_register refuses the brk heap) */
	uint8_t *ring = mmap(NULL, (size_t)maxb * SLOT, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
	if (ring == MAP_FAILED)
		ring = NULL;
	cgck_desc_t *desc = malloc(sizeof(cgck_desc_t) * maxb);
	uint32_t *out = malloc(4 * maxb);
	uint8_t *ver = malloc(maxb);
	double *tt = malloc(sizeof(double) * it), *ph[7];
	for (int k = 0; k < 7; k++)
		ph[k] = malloc(sizeof(double) * it);
	cgck_ctx_t *ctx;
	if (!ring || cgck_ctx_create(0, &ctx))
		return 1;
	memset(ring, 0, (size_t)maxb * SLOT);
	for (int i = 0; i < maxb; i++) {
		uint8_t *ip = ring + (size_t)i * SLOT + L3;
		for (int b = 0; b < len; b++)
			ip[b] = (uint8_t)(i * 7 + b * 13);
		ip[0] = 0x45;
		ip[2] = (uint8_t)(len >> 8);
		ip[3] = (uint8_t)len;
		ip[9] = 17;
		desc[i].frame_off = (uint64_t)i * SLOT;
		desc[i].l3_off = L3;
		desc[i].ip_len = (uint16_t)len;
	}
	if (cgck_host_register(ring, (size_t)maxb * SLOT) || cgck_burst_open(ctx, maxb, (size_t)maxb * 1536, 0)) {
		fprintf(stderr, "srvlat: setup: %s\n", cgck_last_error());
		return 1;
	}
	/* argv[2]: "raw" for CGCK_RAW requests (no header work), "fill" for an
	 * in-place fill (the frames read where they lie in the registered ring,
	 * the fields stored there), else the BSD verify flags (small requests
	 * copy the frames into the request block) */
	const int fill = argc > 2 && !strcmp(argv[2], "fill");
	const uint32_t vf = argc > 2 && !strcmp(argv[2], "raw") ? CGCK_RAW
			    : fill ? CGCK_IP | CGCK_L4 | CGCK_ZERO_FIELDS | CGCK_STORE
				   : CGCK_IP | CGCK_L4 | CGCK_VERIFY | CGCK_V_IP_ZERO_IS_FFFF | CGCK_V_UDP_ZERO_SKIP;
	const int bursts[] = {1, 32, 64, 65, 256, 2048};
	for (unsigned bi = 0; bi < sizeof(bursts) / sizeof(bursts[0]); bi++) {
		const int R = bursts[bi];
		for (int w = 0; w < 50; w++)
			cgck_desc_host(ctx, ring, (size_t)R * SLOT, desc, R, vf, out, ver);
		for (int i = 0; i < it; i++) {
			double a = now();
			if (cgck_desc_host(ctx, ring, (size_t)R * SLOT, desc, R, vf, out, ver)) {
				fprintf(stderr, "srvlat: %s\n", cgck_last_error());
				return 1;
			}
			tt[i] = (now() - a) * 1e6;
			uint64_t d[5], h[2];
			cgck_lab_burst_times(ctx, d, h);
			ph[0][i] = (d[1] - d[0]) / 100.0; /* seen -> block read + checked */
			ph[1][i] = (d[2] - d[1]) / 100.0; /* -> computed (outputs issued) */
			ph[2][i] = (d[3] - d[2]) / 100.0; /* -> release fence done */
			ph[3][i] = (h[1] - h[0]) / 1000.0; /* host post -> done seen */
			ph[4][i] = tt[i] - ph[3][i];       /* host work outside the wait */
			ph[5][i] = d[2] > d[1] ? d[4] / ((d[2] - d[1]) * 10.0) : 0; /* shader clock in GHz */
			ph[6][i] = (double)cgck_lab_burst_body(ctx); /* one-workgroup body call alone, shader clocks */
		}
		printf("{\"pkt_len\": %d, \"burst\": %d, \"us_call\": %.2f, \"us_wait\": %.2f, \"us_host_rest\": %.2f, "
		       "\"us_read\": %.2f, \"us_compute\": %.2f, \"us_release\": %.2f, \"ghz_compute\": %.2f, "
		       "\"body_cycles\": %.0f}\n",
		       len, R, med(tt, it), med(ph[3], it), med(ph[4], it), med(ph[0], it), med(ph[1], it),
		       med(ph[2], it), med(ph[5], it), med(ph[6], it));
		fflush(stdout);
	}
	cgck_burst_close(ctx);
	cgck_host_unregister(ring);
	cgck_ctx_destroy(ctx);
	return 0;
}
