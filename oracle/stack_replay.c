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

/* ---------------------------------------------------------------------- */
/* bsd44 with the packets RX processing builds (round 5)                   */
/* ---------------------------------------------------------------------- */
/*
 * The same bsd44 receive path, carried on past the checksum verdicts to the
 * packets it sends back while it processes a burst:
 *
 *   ip_input.c:82-90    a datagram not for us     -> icmp_error UNREACH_NET;
 *   udp_usrreq.c:98-108 a datagram to a closed port -> icmp_error UNREACH_PORT;
 *   tcp_input.c:86-129, 881-899  a segment with no PCB -> tcp_respond RST;
 *   ip_icmp.c:282-288, 329-352   an echo request -> icmp_reflect (echo reply);
 *   tcp_timer.c:214     keepalive probes at check_timers (tcp_respond from
 *                       the connection's template, tcp_subr.c:52-123).
 *
 * No PCB exists (every port is closed), so every accepted TCP segment draws
 * a RST and every accepted UDP datagram a port unreachable.  The response is
 * built as the reference builds it — io_init_tx_packet hands out the next
 * transmit slot (netmap_init_tx_packet, netmap.c:74-83), or the packet's own
 * pkt_body when the ring is full — and finished by ip_output (ip_output.c:
 * 43-75), every checksum call going through the same function pointers.  The
 * RX frame mutations on the way (NTOHS/NTOHL of the TCP fields, ip_len
 * adjustments, the echo type rewrite, NTOHS of an ICMP error's inner
 * ip_len) are made as the reference makes them, so both rings can be
 * compared byte for byte after a replay.
 */

enum { R_NOTOURS = 5 }; /* ip_input.c:90: answered with icmp_error, not delivered */

/* Transmit side of one replay. */
struct txr {
	uint8_t *slots;     /* the transmit ring: slot k at slots + k * slot */
	uint64_t slot;
	uint32_t cap, used; /* slots in the ring, handed out */
	uint8_t *local;     /* pkt_body of the packets built while the ring was full (2048 B each) */
	uint32_t nlocal;
	uint16_t ip_id;     /* ip_output.c:40, per thread */
	uint32_t laddr_min, laddr_max; /* t_ip_laddr_min/max, host order */
	uint32_t sent[4];   /* RSTs, ICMP errors, echo replies, keepalives */
};

static uint32_t ld32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static void st32(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }
static uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

/* io_init_tx_packet: the IPv4 header's address in the next slot. */
static uint8_t *tx_alloc(struct txr *x)
{
	uint8_t *b = x->used < x->cap ? x->slots + x->slot * x->used++ : x->local + 2048 * (uint64_t)x->nlocal++;
	return b + 14;
}

/* icmp_reflectsrc, ip_icmp.c:52-62. */
static uint32_t reflectsrc(const struct txr *x, uint32_t dst)
{
	uint32_t h = bswap32(dst);
	if (h >= x->laddr_min && h <= x->laddr_max)
		return dst;
	return bswap32(x->laddr_min);
}

/* ip_output.c:43-75 (ip_len host order on entry); t_ip_do_outcksum = 1. */
static void ip_output_r(struct txr *x, uint8_t *ip, in_fn fin, uint64_t *ctr)
{
	static const uint8_t eh[14] = {2, 0, 0, 0, 0, 2, 2, 0, 0, 0, 0, 1, 0x08, 0x00};
	ip[0] = (uint8_t)((ip[0] & 0x0F) | 0x40);    /* :50 ip_v */
	uint16_t off = 0x4000;                         /* :51 IP_DF */
	st16(ip + 4, bswap(x->ip_id++));               /* :52 */
	ip[8] = 64;                                    /* :53 IPDEFTTL */
	ip[1] = 0;                                     /* :54 */
	ip[0] = (uint8_t)((ip[0] & 0xF0) | 5);         /* :55 */
	st16(ip + 2, bswap(ld16(ip + 2)));             /* :58 */
	st16(ip + 6, bswap(off));                      /* :59 */
	st16(ip + 10, 0);                              /* :60 */
	ctr[C_IN_CALLS]++;
	st16(ip + 10, fin(ip, (ip[0] & 15) << 2));     /* :62 ip_cksum */
	memcpy(ip - 14, eh + 6, 6);                    /* :65-67 dhost, shost, type */
	memcpy(ip - 8, eh, 6);
	memcpy(ip - 2, eh + 12, 2);
}

/* icmp_send, ip_icmp.c:68-80. */
static void icmp_send_r(struct txr *x, uint8_t *nip, in_fn fin, uint64_t *ctr)
{
	uint8_t *icp = nip + 20;
	st16(icp + 2, 0);
	ctr[C_IN_CALLS]++;
	st16(icp + 2, fin(icp, ld16(nip + 2) - 20));
	ip_output_r(x, nip, fin, ctr);
}

/* icmp_error, ip_icmp.c:85-154 (type UNREACH; oip's ip_len / ip_off host order). */
static void icmp_error_r(struct txr *x, uint8_t *oip, int code, in_fn fin, uint64_t *ctr)
{
	const uint32_t oiplen = (uint32_t)(oip[0] & 15) << 2;
	if (ld16(oip + 6) & ~(0x2000 | 0x4000))        /* :104 */
		return;
	uint8_t *nip = tx_alloc(x);
	const uint32_t oip_len = ld16(oip + 2);
	const uint32_t icmplen = oiplen + (oip_len < 8 ? oip_len : 8); /* :113 */
	uint8_t *icp = nip + 20;
	icp[0] = 3;                                    /* :119 ICMP_UNREACH */
	st32(icp + 4, 0);                              /* :123 icmp_void */
	icp[1] = (uint8_t)code;                        /* :135 */
	uint8_t *eip = icp + 8;
	memcpy(eip, oip, icmplen);                     /* :137 */
	st16(eip + 2, bswap((uint16_t)(ld16(eip + 2) + oiplen))); /* :138 */
	memcpy(nip, oip, 20);                          /* :142 */
	const uint32_t t = ld32(nip + 16);
	st32(nip + 16, ld32(nip + 12));
	st32(nip + 12, reflectsrc(x, t));
	st16(nip + 2, (uint16_t)(20 + icmplen + 8));   /* :147 */
	nip[0] = (uint8_t)((nip[0] & 0xF0) | 5);
	nip[9] = 1;
	nip[1] = 0;
	nip[8] = 255;                                  /* :151 MAXTTL */
	x->sent[1]++;
	icmp_send_r(x, nip, fin, ctr);
}

/* tcp_template + tcp_respond, tcp_subr.c:52-123.  rcv: the received header
 * (tp == NULL); ka: the connection's addresses and ports (tp != NULL). */
static void tcp_respond_r(struct txr *x, const uint8_t *rcv_ip, const uint8_t *rcv_th, const uint8_t *ka,
			  uint32_t ack, uint32_t seq, int flags, in_fn fin, udp_fn fudp, uint64_t *ctr)
{
	uint8_t *ip = tx_alloc(x), *th = ip + 20;
	ip[0] = 0x45;                                  /* :56-57 (tos, ttl left as the slot had them) */
	st16(ip + 2, bswap(20));                       /* :58 */
	st16(ip + 4, 0);
	st16(ip + 6, 0);
	ip[9] = 6;
	st16(ip + 10, 0);
	if (ka) {                                      /* :63-68 */
		memcpy(ip + 12, ka, 4);
		memcpy(ip + 16, ka + 4, 4);
		memcpy(th, ka + 8, 2);
		memcpy(th + 2, ka + 10, 2);
	}
	st32(th + 4, 0);
	st32(th + 8, 0);
	th[12] = 20 << 2;                              /* :72 th_off */
	th[13] = 0;
	st16(th + 14, 0);
	st16(th + 16, 0);
	st16(th + 18, 0);
	if (!ka) {                                     /* :104-110 */
		memcpy(ip + 12, rcv_ip + 16, 4);
		memcpy(ip + 16, rcv_ip + 12, 4);
		memcpy(th, rcv_th + 2, 2);
		memcpy(th + 2, rcv_th, 2);
	}
	st32(th + 4, bswap32(seq));                    /* :111-113 */
	st32(th + 8, bswap32(ack));
	th[13] = (uint8_t)(flags ? flags : 0x10);
	if (!ka) {
		st16(th + 14, 0);                      /* :114-115 */
	} else {
		uint32_t hiwat, scale;                 /* :117-118 */
		memcpy(&hiwat, ka + 20, 4);
		memcpy(&scale, ka + 24, 4);
		st16(th + 14, bswap((uint16_t)(hiwat >> scale)));
	}
	st16(ip + 2, 40);                              /* :120 (host order) */
	ctr[C_UDP_CALLS]++;
	st16(th + 16, fudp(ip, 20));                   /* :121 tcp_cksum(ip, sizeof(*th)) */
	ip_output_r(x, ip, fin, ctr);
}

/* tcp_input.c:60-129 and 881-899 with no PCB (ip_len host order, minus hlen). */
static int bsd_tcp_input_rsp(struct txr *x, uint8_t *ip, int iphlen, int do_in, in_fn fin, udp_fn fudp,
			     uint64_t *ctr)
{
	int r = bsd_tcp_input(ip, iphlen, do_in, fudp, ctr);
	if (r != R_ACCEPT)
		return r;
	uint8_t *th = ip + iphlen;
	int off = (th[12] & 0xf0) >> 2;                /* :90 */
	if (off < 20 || off > ld16(ip + 2))
		return R_DROP;
	st16(ip + 2, (uint16_t)(ld16(ip + 2) - off));  /* :95 */
	const int flags = th[13];
	st32(th + 4, bswap32(ld32(th + 4)));           /* :106-109 */
	st32(th + 8, bswap32(ld32(th + 8)));
	st16(th + 14, bswap(ld16(th + 14)));
	st16(th + 18, bswap(ld16(th + 18)));
	if (flags & 0x10) {                            /* :891 TH_ACK */
		tcp_respond_r(x, ip, th, NULL, 0, ld32(th + 8), 0x04, fin, fudp, ctr);
	} else {
		if (flags & 0x02)                      /* :894 TH_SYN */
			st16(ip + 2, (uint16_t)(ld16(ip + 2) + 1));
		tcp_respond_r(x, ip, th, NULL, ld32(th + 4) + ld16(ip + 2), 0, 0x04 | 0x10, fin, fudp, ctr);
	}
	x->sent[0]++;
	return R_ACCEPT;
}

/* udp_usrreq.c:53-108 with no PCB. */
static int bsd_udp_input_rsp(struct txr *x, uint8_t *ip, int iphlen, in_fn fin, udp_fn fudp, uint64_t *ctr)
{
	int r = bsd_udp_input(ip, iphlen, fudp, ctr);
	if (r != R_ACCEPT)
		return r;
	st16(ip + 2, (uint16_t)(ld16(ip + 2) + iphlen)); /* :104-105 (save_ip is the same header) */
	icmp_error_r(x, ip, 3, fin, ctr);              /* :106 ICMP_UNREACH_PORT */
	return R_ACCEPT;
}

/* ip_icmp.c:194-288, 329-352 after the checksum verdict. */
static int bsd_icmp_input_rsp(struct txr *x, uint8_t *ip, int hlen, in_fn fin, udp_fn fudp, uint64_t *ctr)
{
	(void)fudp;
	int r = bsd_icmp_input(ip, hlen, fin, ctr);
	if (r != R_ACCEPT)
		return r;
	const int icmplen = ld16(ip + 2);
	uint8_t *icp = ip + hlen;
	const int type = icp[0], code = icp[1];
	if (type > 18)                                 /* :202 ICMP_MAXTYPE */
		return R_ACCEPT;
	int deliver = 0, advise = 0;
	switch (type) {
	case 3:                                        /* UNREACH: codes 0..12 (NEEDFRAG included) */
		deliver = code <= 12;
		break;
	case 11:                                       /* TIMXCEED, PARAMPROB */
	case 12:
		deliver = code <= 1;
		break;
	case 4:                                        /* SOURCEQUENCH */
		deliver = code == 0;
		break;
	case 5:                                        /* REDIRECT: the length check only */
		advise = code <= 3;
		break;
	case 8: {                                      /* :282-288 ECHO -> icmp_reflect */
		icp[0] = 0;
		st16(ip + 2, (uint16_t)(ld16(ip + 2) + hlen));
		uint8_t *nip = tx_alloc(x);
		const int optlen = hlen - 20;
		memcpy(nip, ip, 20);                   /* :341-342 */
		memcpy(nip + 20, ip + hlen, ld16(ip + 2) - hlen);
		const uint32_t t = ld32(nip + 16);
		memcpy(nip + 16, ip + 12, 4);
		st32(nip + 12, reflectsrc(x, t));
		nip[0] = (uint8_t)((nip[0] & 0xF0) | 5);
		nip[8] = 255;
		st16(nip + 2, (uint16_t)(ld16(nip + 2) - optlen));
		x->sent[2]++;
		icmp_send_r(x, nip, fin, ctr);
		return R_ACCEPT;
	}
	default:
		return R_ACCEPT;
	}
	if (deliver || advise) {                       /* :252-256, 291-296 */
		const int advlen = 8 + ((icp[8] & 15) << 2) + 8;
		if (icmplen < 36 || icmplen < advlen || (icp[8] & 15) < 5)
			return R_ACCEPT;
		if (deliver)                           /* :258 NTOHS(icmp_ip.ip_len); no PCB to advise */
			st16(icp + 10, bswap(ld16(icp + 10)));
	}
	return R_ACCEPT;
}

/* ip_input.c:20-112 with the destination check (:82-90). */
static int bsd_ip_input_rsp(struct txr *x, uint8_t *ip, int len, int ip_in, int tcp_in, in_fn fin, udp_fn fudp,
			    uint64_t *ctr)
{
	if (len < 20 || (ip[0] >> 4) != 4)
		return R_DROP;
	int hlen = (ip[0] & 15) << 2;
	if (hlen < 20 || hlen > len)
		return R_DROP;
	uint16_t ip_sum = ld16(ip + 10);
	if (ip_sum == 0)
		ip_sum = 0xffff;
	st16(ip + 10, 0);
	if (ip_in) {
		ctr[C_IN_CALLS]++;
		st16(ip + 10, fin(ip, (ip[0] & 15) << 2));
		if (ld16(ip + 10) != ip_sum) {
			ctr[C_IPS_BADSUM]++;
			return R_DROP_IP;
		}
	}
	st16(ip + 2, bswap(ld16(ip + 2)));
	if (ld16(ip + 2) < hlen)
		return R_DROP;
	st16(ip + 4, bswap(ld16(ip + 4)));
	st16(ip + 6, bswap(ld16(ip + 6)));
	if (len < ld16(ip + 2))
		return R_DROP;
	const uint32_t dst = bswap32(ld32(ip + 16));   /* :82-87 */
	if (dst < x->laddr_min || dst > x->laddr_max) {
		icmp_error_r(x, ip, 0, fin, ctr);      /* :90 ICMP_UNREACH_NET */
		return R_NOTOURS;
	}
	if (ld16(ip + 6) & ~0x4000)
		return R_DROP;
	st16(ip + 2, (uint16_t)(ld16(ip + 2) - hlen));
	switch (ip[9]) {
	case 6:
		return bsd_tcp_input_rsp(x, ip, hlen, tcp_in, fin, fudp, ctr);
	case 17:
		return bsd_udp_input_rsp(x, ip, hlen, fin, fudp, ctr);
	case 1:
		return bsd_icmp_input_rsp(x, ip, hlen, fin, fudp, ctr);
	default:
		return R_ACCEPT;
	}
}

/* One thread_process iteration's receive burst and timers on bsd44, with
 * the packets they send: the burst as oracle_replay_rx, then nka keepalive
 * probes (tcp_timer.c:214; ka: 28-byte records {laddr, faddr, lport, fport
 * (network order), rcv_nxt, snd_una, so_rcv_hiwat, rcv_scale (host)}).
 * txs: {ring slots used, pkt_body packets built, RSTs, ICMP errors, echo
 * replies, keepalives}; *ip_id carries ip_output's counter across calls. */
void oracle_replay_rx_rsp(void *fin, void *fudp, uint8_t *base, const uint8_t *desc12, uint64_t n, int ip_in,
			  int tcp_in, uint8_t *res, uint64_t *ctr, uint8_t *tx_slots, uint64_t tx_slot, uint32_t tx_cap,
			  uint8_t *tx_local, uint32_t laddr_min, uint32_t laddr_max, const uint8_t *ka, uint32_t nka,
			  uint16_t *ip_id, uint32_t *txs)
{
	struct txr x = {tx_slots, tx_slot, tx_cap, 0, tx_local, 0, *ip_id, laddr_min, laddr_max, {0, 0, 0, 0}};
	for (uint64_t k = 0; k < n; k++) {
		uint64_t off;
		uint16_t l3, len;
		memcpy(&off, desc12 + 12 * k, 8);
		memcpy(&l3, desc12 + 12 * k + 8, 2);
		memcpy(&len, desc12 + 12 * k + 10, 2);
		res[k] = (uint8_t)bsd_ip_input_rsp(&x, base + off + l3, len, ip_in, tcp_in, (in_fn)fin, (udp_fn)fudp, ctr);
	}
	for (uint32_t i = 0; i < nka; i++) {           /* check_timers (con-gen.c:524) */
		const uint8_t *r = ka + 28 * (uint64_t)i;
		uint32_t rcv_nxt, snd_una;
		memcpy(&rcv_nxt, r + 12, 4);
		memcpy(&snd_una, r + 16, 4);
		tcp_respond_r(&x, NULL, NULL, r, rcv_nxt, snd_una - 1, 0, (in_fn)fin, (udp_fn)fudp, ctr);
		x.sent[3]++;
	}
	*ip_id = x.ip_id;
	txs[0] = x.used;
	txs[1] = x.nlocal;
	for (int i = 0; i < 4; i++)
		txs[2 + i] = x.sent[i];
}
