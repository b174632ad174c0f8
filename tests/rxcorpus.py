"""Receive-burst corpora for the RX-window tests: frames as a transport hands
them to the stack (an Ethernet header, then `len` bytes from the IPv4
header on, ip_input's `len`), laid out in 2048-byte ring slots with the IPv4
header at +14 (netmap-like).  Checksums are filled the way the reference's
TX path fills them (tcp_output.c:416-418 / udp_usrreq.c:186-190 /
ip_icmp.c:76-77, then ip_output.c:61-64), with the given in_cksum /
udp_cksum (the reference build, or the oracle restatement).
"""
import numpy as np

import cgck

SLOT = 2048
L2 = 14


def be16(p, off, v):
    p[off] = (v >> 8) & 0xFF
    p[off + 1] = v & 0xFF


def le16(p, off, v):
    p[off] = v & 0xFF
    p[off + 1] = (v >> 8) & 0xFF


def frame(rng, ck, proto, l4len, ihl=5, df=True, ttl=64, ulen=None, tcp_off=5, fill=True, pre=None):
    """One IPv4 datagram of ihl*4 + l4len bytes with correct checksums
    (`ck` has in_cksum(buf, off, n) and udp_cksum(buf, off, n)); `pre(p,
    hl)` sets further fields before the checksums are filled."""
    hl = 4 * ihl
    ln = hl + l4len
    p = rng.integers(0, 256, ln, dtype=np.uint8)
    p[0] = 0x40 | ihl
    p[1] = 0
    be16(p, 2, ln)
    p[6], p[7] = (0x40, 0) if df else (0, 0)
    p[8] = ttl
    p[9] = proto
    if proto == 6 and l4len >= 13:
        p[hl + 12] = (tcp_off << 4) | (int(p[hl + 12]) & 0x0F)
    if proto == 17 and l4len >= 6:
        be16(p, hl + 4, l4len if ulen is None else ulen)
    if pre is not None:
        pre(p, hl)
    if fill:
        if proto == 6 and l4len >= 18:
            le16(p, hl + 16, 0)
            le16(p, hl + 16, ck.udp_cksum(p, 0, l4len))
        elif proto == 17 and l4len >= 8:
            le16(p, hl + 6, 0)
            le16(p, hl + 6, ck.udp_cksum(p, 0, l4len if ulen is None else ulen))
        elif proto == 1 and l4len >= 4:
            le16(p, hl + 2, 0)
            le16(p, hl + 2, ck.in_cksum(p, hl, l4len))
        le16(p, 10, 0)
        le16(p, 10, ck.in_cksum(p, 0, hl))
    return p


def corpus(rng, ck, n, clean=False):
    """n frames.  clean: well-formed TCP/UDP/ICMP frames (some corrupted,
    some with Ethernet padding) on which every checksum call the stacks make
    matches a window entry.  Otherwise also the edge shapes: truncated
    frames, options, short headers, other versions, TTL 0, fragments, UDP
    lengths below ip_len, short TCP segments, ICMP below ICMP_ADVLENMIN."""
    out = []
    for i in range(n):
        kind = int(rng.integers(0, 100))
        proto = (6, 6, 6, 17, 1)[i % 5]
        l4 = int(rng.choice([20, 21, 32, 44, 100, 501, 502, 1480]) if proto == 6 else
                 rng.choice([8, 9, 20, 64, 333, 1472]) if proto == 17 else
                 rng.choice([8, 9, 36, 64, 84, 1480]))
        ihl = 5 if i % 7 else int(rng.integers(6, 16))
        if ihl * 4 + l4 > 1500:
            l4 = 1500 - ihl * 4
        p = frame(rng, ck, proto, l4, ihl=ihl)
        if kind < 12:                       # payload bit flip
            j = int(rng.integers(ihl * 4, len(p)))
            p[j] ^= 1 << int(rng.integers(0, 8))
        elif kind < 20:                     # header bit flip (src/dst/ttl/id)
            p[int(rng.choice([4, 5, 8, 12, 15, 19]))] ^= 0x10
        elif kind < 24:                     # wrong L4 field
            fo = {6: 16, 17: 6, 1: 2}[proto]
            p[ihl * 4 + fo] ^= 0x01
        elif kind < 27 and proto == 17:     # "not checksummed" (udp_usrreq.c:86)
            le16(p, ihl * 4 + 6, 0)
        elif kind < 30:                     # wrong IP field
            p[10] ^= 0x80
        if kind >= 30 and kind < 40:        # Ethernet padding past ip_len
            p = np.concatenate([p, rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8)])
        if not clean and kind >= 40 and kind < 70:
            e = kind - 40
            if e < 3:                       # truncated: the frame ends before ip_len
                p = p[:max(20, len(p) - int(rng.integers(1, 30)))]
            elif e < 5:                     # ip_hl < 5
                p[0] = 0x40 | int(rng.integers(0, 5))
            elif e < 7:                     # version 6
                p[0] = 0x60 | (p[0] & 15)
            elif e < 9:                     # TTL 0 (gbtcp drops)
                p[8] = 0
            elif e < 11:                    # fragments (bsd drops after the IP sum, gbtcp bypasses)
                p[6], p[7] = 0x20, 0x10
            elif e < 13 and proto == 17:    # uh_ulen below ip_len: checksum over ulen
                q = frame(rng, ck, 17, l4, ihl=ihl, ulen=max(8, l4 - int(rng.integers(1, 8))))
                p = q
            elif e < 15 and proto == 6:     # TCP segment shorter than its header
                p = frame(rng, ck, 6, int(rng.integers(14, 20)), ihl=ihl)
            elif e < 17 and proto == 1:     # ICMP below ICMP_MINLEN / ICMP_ADVLENMIN
                p = frame(rng, ck, 1, int(rng.integers(2, 36)), ihl=ihl)
            elif e < 19:                    # ip_len below the header length
                be16(p, 2, int(rng.integers(0, ihl * 4)))
            elif e < 21:                    # frame shorter than an IPv4 header
                p = p[:int(rng.integers(0, 20))]
            elif e < 23:                    # other protocol
                p[9] = 47
            elif e < 25 and proto == 6:     # TCP data offset < 5 (gbtcp badoff after the sum)
                p[ihl * 4 + 12] = 0x30
        out.append(p)
    return out


def ring(frames):
    """(ring bytes, DESC_DTYPE descriptors): frame k in slot k at +L2."""
    buf = np.zeros(len(frames) * SLOT + 64, np.uint8)
    desc = np.zeros(len(frames), cgck.DESC_DTYPE)
    for k, p in enumerate(frames):
        o = k * SLOT
        buf[o:o + L2] = (0x02, 0, 0, 0, 0, 1, 0x02, 0, 0, 0, 0, 2, 0x08, 0x00)
        buf[o + L2:o + L2 + len(p)] = p
        desc[k] = (o, L2, len(p))
    return buf, desc


def registered_copy(buf):
    """A copy of `buf` in an anonymous mapping of its own (for
    cgck_host_register, which refuses the brk heap): (owner, view, size)."""
    import mmap
    size = (len(buf) + 4095) // 4096 * 4096
    m = mmap.mmap(-1, size, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    r = np.frombuffer(m, np.uint8)
    r[:len(buf)] = buf
    return m, r, size

LADDR = (0x0A000001, 0x0A000004)   # t_ip_laddr_min/max of the response corpora (10.0.0.1-4)


def rsp_corpus(rng, ck, n, laddr=LADDR):
    """n frames that draw replies from bsd44 with no PCB
    (oracle_replay_rx_rsp): TCP segments of every flag mix to closed ports
    (RST, tcp_input.c:881-899), UDP datagrams to closed ports (port
    unreachable, udp_usrreq.c:98-108), ICMP echo requests (echo reply,
    ip_icmp.c:282-288) and other ICMP types, datagrams for addresses that
    are not ours (net unreachable, ip_input.c:90), fragments; one in eight
    corrupted (payload, header or L4 field), some with uh_ulen below ip_len
    or an ICMP message below ICMP_ADVLENMIN."""
    out = []
    for i in range(n):
        kind = int(rng.integers(0, 100))
        proto = (6, 6, 17, 1)[i % 4]
        ours = kind >= 12
        dst = int(rng.integers(laddr[0], laddr[1] + 1)) if ours else int(rng.integers(0x0B000000, 0x0C000000))
        if proto == 6:
            l4 = int(rng.choice([20, 20, 24, 32, 52, 300, 1460]))
        elif proto == 17:
            l4 = int(rng.choice([8, 9, 20, 64, 512, 1472]))
        else:
            l4 = int(rng.choice([8, 20, 36, 40, 64, 84, 1000]))
        ihl = 5 if i % 9 else int(rng.integers(6, 9))
        if ihl * 4 + l4 > 1500:
            l4 = 1500 - ihl * 4
        tflags = int(rng.choice([0x02, 0x10, 0x12, 0x04, 0x14, 0x18, 0x11, 0x00, 0x01, 0x03]))
        itype, icode = (8, 0) if kind % 3 else (int(rng.choice([3, 3, 11, 12, 4, 5, 0, 13, 30])),
                                                int(rng.integers(0, 16)))

        def pre(p, hl, dst=dst, proto=proto, tflags=tflags, itype=itype, icode=icode):
            p[16], p[17], p[18], p[19] = (dst >> 24) & 255, (dst >> 16) & 255, (dst >> 8) & 255, dst & 255
            if proto == 6 and len(p) >= hl + 14:
                p[hl + 13] = tflags
            if proto == 1 and len(p) >= hl + 2:
                p[hl], p[hl + 1] = itype, icode
                if itype != 8 and len(p) >= hl + 28:     # an inner IPv4 header for the error types
                    p[hl + 8] = 0x45
        ulen = None
        if proto == 17 and kind % 17 == 5:
            ulen = max(8, l4 - int(rng.integers(1, 8)))
        p = frame(rng, ck, proto, l4, ihl=ihl, ulen=ulen, pre=pre, df=kind % 23 != 7)
        if kind % 23 == 7:                  # a fragment (ip_off MF): no error for it, no delivery
            p[6] = 0x20
            le16(p, 10, 0)
            le16(p, 10, ck.in_cksum(p, 0, ihl * 4))
        c = int(rng.integers(0, 8))
        if c == 0:                          # payload bit flip
            j = int(rng.integers(ihl * 4, len(p)))
            p[j] ^= 1 << int(rng.integers(0, 8))
        elif c == 1 and kind % 2:           # header bit flip
            p[int(rng.choice([4, 5, 8, 12, 15]))] ^= 0x10
        elif c == 1:                        # wrong L4 field
            p[ihl * 4 + {6: 16, 17: 6, 1: 2}[proto]] ^= 0x01
        out.append(p)
    return out


def pool(frames, tx_slots):
    """One registered-style pool of 2048-byte slots, as a netmap pool holds
    both rings: receive frame k in slot 2k at +14, transmit slot j at slot
    2j + 1 while j < len(frames), then after them.  Returns (pool bytes,
    DESC_DTYPE descriptors, transmit base offset, transmit stride)."""
    nrx = len(frames)
    nslots = 2 * max(nrx, tx_slots) + 1
    buf = np.zeros(nslots * SLOT, np.uint8)
    desc = np.zeros(nrx, cgck.DESC_DTYPE)
    for k, p in enumerate(frames):
        o = 2 * k * SLOT
        buf[o:o + L2] = (0x02, 0, 0, 0, 0, 1, 0x02, 0, 0, 0, 0, 2, 0x08, 0x00)
        buf[o + L2:o + L2 + len(p)] = p
        desc[k] = (o, L2, len(p))
    return buf, desc, SLOT, 2 * SLOT
