/*
 * stack_replay.c — TEST INFRASTRUCTURE ONLY.
 *
 * Restates the receive-side call sequences of the reference's two stacks
 * around the checksum unit, up to and including their checksum verdicts:
 *
 *   bsd44: ip_input.c:20-112, tcp_input.c:60-85, udp_usrreq.c:53-94,
 *          ip_icmp.c:160-193 (counters netstat.h:40,103,129,150);
 *   gbtcp: inet.c:275-352 (ip_in) and 118-159 (tcp_in).
 *
 * Every header mutation the reference makes on the way (the zeroed and
 * rewritten checksum fields, NTOHS of ip_len/ip_id/ip_off, ip_len -= hlen,
 * gbtcp's restored fields) is made the same way, so the bytes after a replay
 * can be compared.  The checksum calls go through function pointers: the
 * tests replay one copy of a burst with the reference's own in_cksum /
 * udp_cksum (oracle/_ref) and another with libcgck.so's drop-in symbols
 * inside an RX window (cgck_rx_begin), and compare outcomes, counter
 * increments and bytes.  Only tests/ load this.
 */
#include <stdint.h>
#include <string.h>

typedef uint16_t (*in_fn)(void *, int);
typedef uint16_t (*udp_fn)(void *, int);

/* Outcome of one frame. */
enum {
	R_ACCEPT = 0,  /* passed every check this replay covers */
	R_DROP = 1,    /* dropped by a length / header check (no checksum verdict) */
	R_DROP_IP = 2, /* dropped on the IP header checksum */
	R_DROP_L4 = 3, /* dropped on the TCP / UDP / ICMP checksum */
	R_BYPASS = 4,  /* gbtcp IN_BYPASS (fragments, other protocols) */
};

/* Counter slots. */
enum {
	C_IPS_BADSUM = 0,     /* ipstat.ips_badsum       (ip_input.c:53, inet.c:324)  */
	C_TCPS_RCVBADSUM = 1, /* tcpstat.tcps_rcvbadsum  (tcp_input.c:80, inet.c:147) */
	C_UDPS_BADSUM = 2,    /* udpstat.udps_badsum     (udp_usrreq.c:91)            */
	C_ICPS_CHECKSUM = 3,  /* icmpstat.icps_checksum  (ip_icmp.c:191)              */
	C_IN_CALLS = 4,       /* in_cksum calls made (ip_cksum included)              */
	C_UDP_CALLS = 5,      /* udp_cksum calls made (tcp_cksum included)            */
};

static uint16_t ld16(const uint8_t *p) { uint16_t v; memcpy(&v, p, 2); return v; }
static void st16(uint8_t *p, uint16_t v) { memcpy(p, &v, 2); }
static uint16_t bswap(uint16_t v) { return (uint16_t)(v << 8 | v >> 8); }

/* ---------------------------------------------------------------------- */
/* bsd44                                                                   */
/* ---------------------------------------------------------------------- */

/* tcp_input.c:60-85 (ip->ip_len is host order and already minus hlen). */
static int bsd_tcp_input(uint8_t *ip, int iphlen, int do_in, udp_fn fudp, uint64_t *ctr)
{
	uint8_t *th = ip + iphlen;
	if (ld16(ip + 2) < 20)            /* :67 sizeof(struct tcp_hdr) */
		return R_DROP;
	int th_sum = ld16(th + 16);       /* :75 */
	st16(th + 16, 0);
	if (do_in) {
		ctr[C_UDP_CALLS]++;
		st16(th + 16, fudp(ip, ld16(ip + 2)));   /* :78 tcp_cksum(ip, ip->ip_len) */
		if (th_sum != ld16(th + 16)) {
			ctr[C_TCPS_RCVBADSUM]++;
			if (do_in > 1)
				return R_DROP_L4;
		}
	}
	return R_ACCEPT;
}

/* udp_usrreq.c:53-94 (udpcksum = 1, :44). */
static int bsd_udp_input(uint8_t *ip, int iphlen, udp_fn fudp, uint64_t *ctr)
{
	int ip_len = ld16(ip + 2);
	if (ip_len < 8)                   /* :65 sizeof(struct udp_hdr) */
		return R_DROP;
	uint8_t *uh = ip + iphlen;
	int len = bswap(ld16(uh + 4));    /* :73 ntohs(uh_ulen) */
	if (ip_len != len && len > ip_len)
		return R_DROP;
	if (ld16(uh + 6)) {               /* :86 */
		int uh_sum = ld16(uh + 6);
		st16(uh + 6, 0);
		ctr[C_UDP_CALLS]++;
		st16(uh + 6, fudp(ip, len));  /* :89 */
		if (ld16(uh + 6) != uh_sum) {
			ctr[C_UDPS_BADSUM]++;
			return R_DROP_L4;
		}
	}
	return R_ACCEPT;
}

/* ip_icmp.c:160-193. */
static int bsd_icmp_input(uint8_t *ip, int hlen, in_fn fin, uint64_t *ctr)
{
	int icmplen = ld16(ip + 2);       /* :170 */
	if (icmplen < 8)                  /* :177 ICMP_MINLEN */
		return R_DROP;
	int i = icmplen < 36 ? icmplen : 36; /* :181 ICMP_ADVLENMIN = 8 + 20 + 8 */
	if (ld16(ip + 2) < i)
		return R_DROP;
	uint8_t *icp = ip + hlen;
	int icmp_cksum = ld16(icp + 2);   /* :187 */
	st16(icp + 2, 0);
	ctr[C_IN_CALLS]++;
	st16(icp + 2, fin(icp, icmplen)); /* :189 */
	if (ld16(icp + 2) != icmp_cksum) {
		ctr[C_ICPS_CHECKSUM]++;
		return R_DROP_L4;
	}
	return R_ACCEPT;
}

/* ip_input.c:20-112; every destination counts as ours (:82-87). */
static int bsd_ip_input(uint8_t *ip, int len, int ip_in, int tcp_in, in_fn fin, udp_fn fudp, uint64_t *ctr)
{
	if (len < 20)                     /* :28 */
		return R_DROP;
	if ((ip[0] >> 4) != 4)            /* :32 ip_v */
		return R_DROP;
	int hlen = (ip[0] & 15) << 2;     /* :36 */
	if (hlen < 20 || hlen > len)      /* :37, :41 */
		return R_DROP;
	uint16_t ip_sum = ld16(ip + 10);  /* :45-49 */
	if (ip_sum == 0)
		ip_sum = 0xffff;
	st16(ip + 10, 0);
	if (ip_in) {
		ctr[C_IN_CALLS]++;
		st16(ip + 10, fin(ip, (ip[0] & 15) << 2)); /* :51 ip_cksum(ip) */
		if (ld16(ip + 10) != ip_sum) {
			ctr[C_IPS_BADSUM]++;
			return R_DROP_IP;     /* :54 any nonzero flag drops */
		}
	}
	st16(ip + 2, bswap(ld16(ip + 2))); /* :63 NTOHS(ip_len) */
	if (ld16(ip + 2) < hlen)
		return R_DROP;
	st16(ip + 4, bswap(ld16(ip + 4))); /* :68-69 */
	st16(ip + 6, bswap(ld16(ip + 6)));
	if (len < ld16(ip + 2))           /* :76 */
		return R_DROP;
	if (ld16(ip + 6) & ~0x4000)       /* :94 ip_off & ~IP_DF */
		return R_DROP;
	st16(ip + 2, (uint16_t)(ld16(ip + 2) - hlen)); /* :98 */
	switch (ip[9]) {
	case 6:
		return bsd_tcp_input(ip, hlen, tcp_in, fudp, ctr);
	case 17:
		return bsd_udp_input(ip, hlen, fudp, ctr);
	case 1:
		return bsd_icmp_input(ip, hlen, fin, ctr);
	default:
		return R_ACCEPT;
	}
}

/* ---------------------------------------------------------------------- */
/* gbtcp (the toy stack)                                                  */
/* ---------------------------------------------------------------------- */

/* inet.c:118-159; rem = bytes after the IP header, payload = total - ih_len. */
static int toy_tcp_in(uint8_t *ip, int ih_len, int rem, int payload, int do_in, udp_fn fudp, uint64_t *ctr)
{
	if (rem < 20)                     /* :123 */
		return R_DROP;
	uint8_t *th = ip + ih_len;
	int th_len = (th[12] & 0xf0) >> 2; /* :128 TCP_HDR_LEN */
	if (rem < th_len)
		return R_DROP;
	int cksum = ld16(th + 16);        /* :142 */
	st16(th + 16, 0);
	if (do_in) {
		ctr[C_UDP_CALLS]++;
		int tmp = fudp(ip, payload);  /* :145 */
		if (cksum != tmp) {
			ctr[C_TCPS_RCVBADSUM]++;
			if (do_in > 1)
				return R_DROP_L4; /* the field stays 0 */
		}
	}
	st16(th + 16, (uint16_t)cksum);   /* :153 */
	if (th_len < 20)                  /* :154 */
		return R_DROP;
	return R_ACCEPT;
}

/* inet.c:275-352; rem = frame bytes after the Ethernet header. */
static int toy_ip_in(uint8_t *ip, int rem, int ip_in, int tcp_in, in_fn fin, udp_fn fudp, uint64_t *ctr)
{
	if (rem < 20)                     /* :282 */
		return R_DROP;
	if (ip[8] < 1)                    /* :287 ih_ttl */
		return R_DROP;
	if (ld16(ip + 6) & 0xFF3F)        /* :293 IP4_FRAG_MASK on the raw field */
		return R_BYPASS;
	int ih_len = (ip[0] & 15) << 2;   /* :298 IP4_HDR_LEN */
	if (ih_len < 20 || rem < ih_len)  /* :299, :303 */
		return R_DROP;
	rem -= ih_len;                    /* :307 SHIFT */
	int total_len = bswap(ld16(ip + 2)); /* :308 */
	if (total_len < ih_len)
		return R_DROP;
	int payload = (uint16_t)(total_len - ih_len); /* :313 (u16 field) */
	if (payload > rem)
		return R_DROP;
	int proto = ip[9];
	int cksum = ld16(ip + 10);        /* :319 */
	st16(ip + 10, 0);
	if (ip_in) {
		ctr[C_IN_CALLS]++;
		int tmp = fin(ip, (ip[0] & 15) << 2); /* :322 ip_cksum */
		if (tmp != cksum) {
			ctr[C_IPS_BADSUM]++;
			if (ip_in > 1)
				return R_DROP_IP; /* the field stays 0 */
		}
	}
	st16(ip + 10, (uint16_t)cksum);   /* :330 */
	switch (proto) {
	case 17:
		return rem < 8 ? R_DROP : R_ACCEPT; /* :333 */
	case 6:
		return toy_tcp_in(ip, ih_len, rem, payload, tcp_in, fudp, ctr);
	case 1:
		return R_ACCEPT; /* icmp4_in (:161-273) checks no checksum */
	default:
		return R_BYPASS;
	}
}

/* One burst: frame k's IPv4 header at base + desc[k].frame_off + l3_off,
 * with desc[k].ip_len bytes after it (the `len` ip_input gets from
 * bsd_eth_in, if_ether.c:161; gbtcp's inp_rem after the Ethernet SHIFT).
 * stack 0 = bsd44, 1 = gbtcp; ip_in / tcp_in = t_ip_do_incksum /
 * t_tcp_do_incksum (0, 1, 2; con-gen.c:733-736).  Outcomes per frame into
 * `res`; counter increments added to ctr[6]. */
void oracle_replay_rx(void *fin, void *fudp, uint8_t *base, const uint8_t *desc12, uint64_t n, int stack,
		      int ip_in, int tcp_in, uint8_t *res, uint64_t *ctr)
{
	for (uint64_t k = 0; k < n; k++) {
		uint64_t off;
		uint16_t l3, len;
		memcpy(&off, desc12 + 12 * k, 8);
		memcpy(&l3, desc12 + 12 * k + 8, 2);
		memcpy(&len, desc12 + 12 * k + 10, 2);
		uint8_t *ip = base + off + l3;
		res[k] = (uint8_t)(stack ? toy_ip_in(ip, len, ip_in, tcp_in, (in_fn)fin, (udp_fn)fudp, ctr)
				      : bsd_ip_input(ip, len, ip_in, tcp_in, (in_fn)fin, (udp_fn)fudp, ctr));
	}
}
