/*
 * rss_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of con-gen's Toeplitz RSS hash (subr.c:482-530) and of the
 * dst-cache loop that calls it (thread_init_dst_cache, con-gen.c:291-360).
 * It is the referee for the gfx950 kernels in con-gen_amd/csrc/cgck_rss.hip
 * and the "port" CPU baseline of that row.  Only tests/, bench.py's
 * cpu_baseline leg and tests/golden/make_golden.py load it; libcgck.so never
 * links or calls it.
 *
 * Pinning: checked against the reference's own toeplitz_hash / rss_hash4
 * compiled from /root/reference (oracle/build_ref.sh -> oracle/_ref/
 * libref_rss.so) through the committed fixtures in tests/golden/rss.json and
 * the published Microsoft RSS verification vectors for the default key
 * (freebsd_rss_key, subr.c:29-35); the dst-cache loop is run with either
 * hash (this file's or the reference build's) through a function pointer.
 */
#include <stdint.h>
#include <string.h>
#include <arpa/inet.h>

/* subr.c:482-502.  A 32-bit window slides along the key one bit per data
 * bit; it starts as key[0..3] and takes in bit (7-b) of key[i+4] while
 * i+4 < key_size, zeros after.  Every set data bit (MSB first) XORs the
 * window into the result. */
uint32_t oracle_toeplitz_hash(const uint8_t *data, int cnt, const uint8_t *key, int key_size)
{
	uint32_t win = (uint32_t)key[0] << 24 | (uint32_t)key[1] << 16 | (uint32_t)key[2] << 8 | key[3];
	uint32_t h = 0;
	for (int i = 0; i < cnt; i++) {
		const uint8_t next = i + 4 < key_size ? key[i + 4] : 0;
		for (int b = 7; b >= 0; b--) {
			if ((data[i] >> b) & 1)
				h ^= win;
			win = (win << 1) | ((next >> b) & 1);
		}
	}
	return h;
}

/* subr.c:506-530.  Data = {faddr, laddr, fport, lport} as stored (network
 * order), 12 bytes; the hash is masked to 7 bits. */
uint32_t oracle_rss_hash4(uint32_t laddr, uint32_t faddr, uint16_t lport, uint16_t fport,
			  const uint8_t *key, int key_size)
{
	uint8_t d[12];
	memcpy(d, &faddr, 4);
	memcpy(d + 4, &laddr, 4);
	memcpy(d + 8, &fport, 2);
	memcpy(d + 10, &lport, 2);
	return oracle_toeplitz_hash(d, 12, key, key_size) & 0x7f;
}

/* Batch referee mirroring cgck_toeplitz (include/cgck.h). */
void oracle_toeplitz_batch(const uint8_t *data, uint64_t n, uint64_t stride, uint32_t cnt,
			   const uint8_t *key, int key_size, uint32_t mask, uint32_t *out)
{
	for (uint64_t k = 0; k < n; k++)
		out[k] = oracle_toeplitz_hash(data + k * stride, (int)cnt, key, key_size) & mask;
}

/* struct ip_socket's dst fields as cgck_dst_entry_t lays them out. */
struct dst_entry {
	uint32_t laddr, faddr;
	uint16_t lport, fport;
	uint32_t hash;
};

typedef uint32_t (*rss_fn)(uint32_t, uint32_t, uint16_t, uint16_t, const uint8_t *, int);

#define EPH_MIN 5000u   /* subr.h:62 */
#define EPH_MAX 65535u  /* subr.h:63 */
#define NEPH (EPH_MAX - EPH_MIN + 1)

/* con-gen.c:291-360 (without the allocation and the concurrency panic,
 * which stay with the caller).  Returns the entries written. */
uint32_t oracle_dst_cache(uint32_t laddr_min, uint32_t laddr_max, uint32_t faddr_min, uint32_t faddr_max,
			  uint16_t fport, uint8_t queue_num, uint8_t queue_id, const uint8_t *key,
			  int key_size, void *hash_fn, struct dst_entry *out, uint32_t cap)
{
	rss_fn hash = hash_fn ? (rss_fn)hash_fn : oracle_rss_hash4;
	/* :314-315, 32-bit unsigned product */
	const uint32_t total = (laddr_max - laddr_min + 1u) * (faddr_max - faddr_min + 1u) * NEPH;
	uint32_t la = laddr_min, fa = faddr_min, lp = EPH_MIN;
	uint32_t got = 0;
	for (uint64_t i = 0; i < total; i++) {
		const uint32_t laddr = htonl(la), faddr = htonl(fa);
		const uint16_t lport = htons((uint16_t)lp);
		/* :320-333 advance: faddr fastest, then lport, then laddr */
		if (fa < faddr_max) {
			fa++;
		} else {
			fa = faddr_min;
			if (lp < EPH_MAX) {
				lp++;
			} else {
				lp = EPH_MIN;
				la = la < laddr_max ? la + 1 : laddr_min;
			}
		}
		/* :337-342 RSS filter */
		if (queue_id < 128 && queue_num > 1) {
			uint32_t h = hash(laddr, faddr, lport, fport, key, key_size);
			if (h % queue_num != queue_id)
				continue;
		}
		/* :344-353 */
		struct dst_entry *e = out + got;
		e->laddr = laddr;
		e->faddr = faddr;
		e->lport = lport;
		e->fport = fport;
		e->hash = faddr ^ (faddr >> 16) ^ ntohs(lport ^ fport); /* SO_HASH, subr.h:179-180 */
		if (++got == cap)
			break;
	}
	return got;
}

void *oracle_fn_rss_hash4(void) { return (void *)oracle_rss_hash4; }
