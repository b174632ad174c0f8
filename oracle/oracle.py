"""ctypes loader for the oracle — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  It exposes two referees:

* ``port()``: the clean C restatement in ``oracle/cksum_oracle.c`` (always
  built by ``make -C oracle``);
* ``reference()``: the reference's own checksum unit (subr.c:119-223) built by
  ``oracle/build_ref.sh`` into ``oracle/_ref/libref_cksum.so`` — ``None`` when
  that build is absent (no /root/reference at build time).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PORT_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libref_cksum.so")
REF_RSS_SO = os.path.join(HERE, "_ref", "libref_rss.so")

DST_DTYPE = np.dtype([("laddr", "<u4"), ("faddr", "<u4"), ("lport", "<u2"), ("fport", "<u2"),
                      ("hash", "<u4")])   # cgck_dst_entry_t

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)


def _ptr(a, t=_u8p):
    return a.ctypes.data_as(t)


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


class Port:
    """The C restatement (oracle/cksum_oracle.c)."""

    def __init__(self, path=PORT_SO):
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        self.lib = L
        L.oracle_in_cksum.restype = ctypes.c_uint16
        L.oracle_in_cksum.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.oracle_udp_cksum.restype = ctypes.c_uint16
        L.oracle_udp_cksum.argtypes = [ctypes.c_void_p, ctypes.c_int]
        for name in ("oracle_bsd_ip_input_verify", "oracle_toy_ip_verify"):
            getattr(L, name).restype = ctypes.c_int
            getattr(L, name).argtypes = [ctypes.c_void_p]
        for name in ("oracle_bsd_tcp_input_verify", "oracle_bsd_udp_input_verify",
                     "oracle_toy_tcp_verify"):
            getattr(L, name).restype = ctypes.c_int
            getattr(L, name).argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.oracle_ip_output_fill.argtypes = [ctypes.c_void_p]
        L.oracle_tcp_output_fill.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.oracle_packet.restype = ctypes.c_uint32
        L.oracle_packet.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, _u32p]
        L.oracle_batch_strided.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                           ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                           ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_batch_desc.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                        ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_splitmix64.restype = ctypes.c_uint64
        L.oracle_splitmix64.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_stream_bytes.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                          ctypes.c_uint64]
        L.oracle_stamp_header.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        L.oracle_synth_packet.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                          ctypes.c_uint32, ctypes.c_uint64]
        L.oracle_imix_desc.argtypes = [ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                       ctypes.POINTER(ctypes.c_uint16)]
        L.oracle_cpu_bench.restype = ctypes.c_double
        L.oracle_cpu_bench.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                       ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_check_synth_strided.restype = ctypes.c_uint64
        L.oracle_check_synth_strided.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                                 ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
                                                 ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_check_synth_imix.restype = ctypes.c_uint64
        L.oracle_check_synth_imix.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                              ctypes.c_void_p, ctypes.c_uint64,
                                              ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_check_synth_ring.restype = ctypes.c_uint64
        L.oracle_check_synth_ring.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                              ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64,
                                              ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_fn_in_cksum.restype = ctypes.c_void_p
        L.oracle_fn_udp_cksum.restype = ctypes.c_void_p
        # Toeplitz RSS (oracle/rss_oracle.c)
        L.oracle_toeplitz_hash.restype = ctypes.c_uint32
        L.oracle_toeplitz_hash.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        L.oracle_rss_hash4.restype = ctypes.c_uint32
        L.oracle_rss_hash4.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint16,
                                       ctypes.c_uint16, ctypes.c_void_p, ctypes.c_int]
        L.oracle_toeplitz_batch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                            ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int,
                                            ctypes.c_uint32, ctypes.c_void_p]
        L.oracle_dst_cache.restype = ctypes.c_uint32
        L.oracle_dst_cache.argtypes = [ctypes.c_uint32] * 4 + [ctypes.c_uint16, ctypes.c_uint8,
                                       ctypes.c_uint8, ctypes.c_void_p, ctypes.c_int,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
        L.oracle_fn_rss_hash4.restype = ctypes.c_void_p
        # RX call-sequence replay (oracle/stack_replay.c)
        L.oracle_replay_rx.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_replay_rx_rsp.argtypes = ([ctypes.c_void_p] * 4 + [ctypes.c_uint64, ctypes.c_int, ctypes.c_int]
                                           + [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_uint32,
                                           ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                           ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p])

    # -- pure functions (subr.c:186-195, 212-223) --
    def in_cksum(self, buf, off=0, n=None):
        """in_cksum(buf+off, n) on a numpy uint8 array."""
        if n is None:
            n = len(buf) - off
        return self.lib.oracle_in_cksum(buf.ctypes.data + off, n)

    def udp_cksum(self, buf, off, n):
        return self.lib.oracle_udp_cksum(buf.ctypes.data + off, n)

    def fn_pointers(self):
        return self.lib.oracle_fn_in_cksum(), self.lib.oracle_fn_udp_cksum()

    # -- batch referees (mirror include/cgck.h flags) --
    def batch_strided(self, base, n, stride, l3_off, ip_len, flags):
        out = np.zeros(n, np.uint32)
        ver = np.zeros(n, np.uint8)
        self.lib.oracle_batch_strided(base.ctypes.data, n, stride, l3_off, ip_len, flags,
                                      out.ctypes.data, ver.ctypes.data)
        return out, ver

    def batch_desc(self, base, desc12, n, flags):
        out = np.zeros(n, np.uint32)
        ver = np.zeros(n, np.uint8)
        self.lib.oracle_batch_desc(base.ctypes.data, desc12.ctypes.data, n, flags,
                                   out.ctypes.data, ver.ctypes.data)
        return out, ver

    # -- synthetic input --
    def stream_bytes(self, off, n, seed):
        out = np.empty(n, np.uint8)
        self.lib.oracle_stream_bytes(out.ctypes.data, off, n, seed)
        return out

    def synth_packet(self, k, stride, ip_len, seed):
        out = np.empty(ip_len, np.uint8)
        self.lib.oracle_synth_packet(out.ctypes.data, k, stride, ip_len, seed)
        return out

    def stamp_header(self, buf, off, ip_len):
        self.lib.oracle_stamp_header(buf.ctypes.data + off, ip_len)

    @staticmethod
    def stamp_strided(buf, n, stride, ip_len):
        """oracle_stamp_header on packets k*stride, k < n, vectorised."""
        v = buf[:n * stride].reshape(n, stride)
        v[:, 0] = 0x45
        v[:, 1] = 0
        v[:, 2] = (ip_len >> 8) & 0xFF
        v[:, 3] = ip_len & 0xFF
        v[:, 9] = 6
        v[:, 10:12] = 0
        if ip_len >= 38:
            v[:, 36:38] = 0

    def imix_desc(self, k):
        off = ctypes.c_uint64()
        ln = ctypes.c_uint16()
        self.lib.oracle_imix_desc(k, ctypes.byref(off), ctypes.byref(ln))
        return off.value, ln.value

    def check_synth_strided(self, n, stride, ip_len, seed, flags, out, every=1):
        """(mismatches, packets checked) of device results `out` vs the referee."""
        chk = ctypes.c_uint64()
        bad = self.lib.oracle_check_synth_strided(n, stride, ip_len, seed, flags, out.ctypes.data,
                                                  every, ctypes.byref(chk))
        return bad, chk.value

    def check_synth_imix(self, n, seed, flags, out, every=1):
        chk = ctypes.c_uint64()
        bad = self.lib.oracle_check_synth_imix(n, seed, flags, out.ctypes.data, every,
                                               ctypes.byref(chk))
        return bad, chk.value

    def check_synth_ring(self, n, stride, l3_off, seed, flags, out, every=1):
        """IMIX frames in ring slots (cgck_synth_imix_ring) vs the referee."""
        chk = ctypes.c_uint64()
        bad = self.lib.oracle_check_synth_ring(n, stride, l3_off, seed, flags, out.ctypes.data, every,
                                               ctypes.byref(chk))
        return bad, chk.value

    # -- Toeplitz RSS (subr.c:482-530, con-gen.c:291-360) --
    def toeplitz_hash(self, data, key, cnt=None, key_size=None):
        data = np.ascontiguousarray(data, np.uint8)
        key = np.ascontiguousarray(key, np.uint8)
        return self.lib.oracle_toeplitz_hash(data.ctypes.data, len(data) if cnt is None else cnt,
                                             key.ctypes.data, len(key) if key_size is None else key_size)

    def rss_hash4(self, laddr, faddr, lport, fport, key, key_size=None):
        key = np.ascontiguousarray(key, np.uint8)
        return self.lib.oracle_rss_hash4(laddr, faddr, lport, fport, key.ctypes.data,
                                         len(key) if key_size is None else key_size)

    def toeplitz_batch(self, data, n, stride, cnt, key, mask=0xFFFFFFFF, key_size=None):
        key = np.ascontiguousarray(key, np.uint8)
        out = np.zeros(n, np.uint32)
        self.lib.oracle_toeplitz_batch(data.ctypes.data, n, stride, cnt, key.ctypes.data,
                                       len(key) if key_size is None else key_size, mask,
                                       out.ctypes.data)
        return out

    def dst_cache(self, laddr_min, laddr_max, faddr_min, faddr_max, fport, queue_num, queue_id,
                  key, cap, hash_fn=None, key_size=None):
        """con-gen.c:291-360 restated; hash_fn = a C rss_hash4 pointer (None:
        this file's).  Returns a DST_DTYPE array of the entries written."""
        key = np.ascontiguousarray(key, np.uint8)
        out = np.zeros(cap, DST_DTYPE)
        got = self.lib.oracle_dst_cache(laddr_min, laddr_max, faddr_min, faddr_max, fport,
                                        queue_num, queue_id, key.ctypes.data,
                                        len(key) if key_size is None else key_size, hash_fn,
                                        out.ctypes.data, cap)
        return out[:got]

    def fn_rss_hash4(self):
        return self.lib.oracle_fn_rss_hash4()

    # outcome codes and counter slots of oracle_replay_rx (oracle/stack_replay.c)
    R_ACCEPT, R_DROP, R_DROP_IP, R_DROP_L4, R_BYPASS = range(5)
    COUNTERS = ("ips_badsum", "tcps_rcvbadsum", "udps_badsum", "icps_checksum", "in_calls", "udp_calls")

    def replay_rx(self, fin, fudp, base, desc12, n, stack, ip_in, tcp_in):
        """Replay the reference stack's RX call sequence (stack 0 bsd44, 1
        gbtcp) over a burst, with the given in_cksum / udp_cksum pointers.
        Mutates `base` as the reference does; returns (outcomes, counters)."""
        res = np.zeros(max(n, 1), np.uint8)
        ctr = np.zeros(6, np.uint64)
        self.lib.oracle_replay_rx(fin, fudp, base.ctypes.data, desc12.ctypes.data, n, stack, ip_in, tcp_in,
                                  res.ctypes.data, ctr.ctypes.data)
        return res[:n], ctr

    R_NOTOURS = 5    # oracle_replay_rx_rsp: ip_input.c:90, answered with icmp_error
    KA_DTYPE = np.dtype([("laddr", "<u4"), ("faddr", "<u4"), ("lport", "<u2"), ("fport", "<u2"),
                         ("rcv_nxt", "<u4"), ("snd_una", "<u4"), ("hiwat", "<u4"), ("scale", "<u4")])

    def replay_rx_rsp(self, fin, fudp, base, desc12, n, ip_in, tcp_in, tx, slot, cap, local, laddr, ka, ip_id):
        """bsd44's receive burst plus the packets it sends back (RSTs, ICMP
        unreachables, echo replies) and nka keepalives from check_timers,
        built into the transmit ring `tx` (cap slots of `slot` bytes; packets
        built while it is full go to `local`, 2048 B each).  Returns
        (outcomes, counters, txs, ip_id): txs = [slots used, pkt_body packets,
        RSTs, ICMP errors, echo replies, keepalives]."""
        res = np.zeros(max(n, 1), np.uint8)
        ctr = np.zeros(6, np.uint64)
        txs = np.zeros(6, np.uint32)
        idc = ctypes.c_uint16(ip_id)
        ka = np.zeros(0, self.KA_DTYPE) if ka is None else ka
        self.lib.oracle_replay_rx_rsp(fin, fudp, base.ctypes.data, desc12.ctypes.data, n, ip_in, tcp_in,
                                      res.ctypes.data, ctr.ctypes.data, tx.ctypes.data, slot, cap,
                                      local.ctypes.data, laddr[0], laddr[1], ka.ctypes.data, len(ka),
                                      ctypes.byref(idc), txs.ctypes.data)
        return res[:n], ctr, txs, idc.value

    def cpu_bench(self, fin, fudp, base, n, stride, ip_len, threads=1, reps=1):
        sink = ctypes.c_uint64()
        sec = self.lib.oracle_cpu_bench(fin, fudp, base.ctypes.data, n, stride, ip_len,
                                        threads, reps, ctypes.byref(sink))
        return sec, sink.value


class Reference:
    """The reference's own subr.c checksum unit (oracle/_ref, built from /root/reference)."""

    def __init__(self, path=REF_SO):
        L = ctypes.CDLL(path)
        self.lib = L
        L.in_cksum.restype = ctypes.c_uint16
        L.in_cksum.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.udp_cksum.restype = ctypes.c_uint16
        L.udp_cksum.argtypes = [ctypes.c_void_p, ctypes.c_int]

    def in_cksum(self, buf, off=0, n=None):
        if n is None:
            n = len(buf) - off
        return self.lib.in_cksum(buf.ctypes.data + off, n)

    def udp_cksum(self, buf, off, n):
        return self.lib.udp_cksum(buf.ctypes.data + off, n)

    def fn_pointers(self):
        return (ctypes.cast(self.lib.in_cksum, ctypes.c_void_p).value,
                ctypes.cast(self.lib.udp_cksum, ctypes.c_void_p).value)


class ReferenceRss:
    """The reference's own Toeplitz unit: freebsd_rss_key, toeplitz_hash and
    rss_hash4 (subr.c:29-35, 482-530), built into oracle/_ref/libref_rss.so."""

    def __init__(self, path=REF_RSS_SO):
        L = ctypes.CDLL(path)
        self.lib = L
        L.toeplitz_hash.restype = ctypes.c_uint32
        L.toeplitz_hash.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        L.rss_hash4.restype = ctypes.c_uint32
        L.rss_hash4.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint16, ctypes.c_uint16,
                                ctypes.c_void_p, ctypes.c_int]
        self.key = np.frombuffer((ctypes.c_uint8 * 40).in_dll(L, "freebsd_rss_key"), np.uint8).copy()

    def toeplitz_hash(self, data, key, cnt=None, key_size=None):
        data = np.ascontiguousarray(data, np.uint8)
        key = np.ascontiguousarray(key, np.uint8)
        return self.lib.toeplitz_hash(data.ctypes.data, len(data) if cnt is None else cnt,
                                      key.ctypes.data, len(key) if key_size is None else key_size)

    def rss_hash4(self, laddr, faddr, lport, fport, key, key_size=None):
        key = np.ascontiguousarray(key, np.uint8)
        return self.lib.rss_hash4(laddr, faddr, lport, fport, key.ctypes.data,
                                  len(key) if key_size is None else key_size)

    def fn_rss_hash4(self):
        return ctypes.cast(self.lib.rss_hash4, ctypes.c_void_p).value


def reference_rss():
    """The reference's RSS build, or None where it was not built."""
    if not os.path.exists(REF_RSS_SO):
        return None
    return ReferenceRss()


_port = None


def port():
    global _port
    if _port is None:
        _port = Port()
    return _port


def reference():
    """The reference build, or None where it was not built (e.g. on the GPU box
    when /root/reference was absent at build time)."""
    if not os.path.exists(REF_SO):
        return None
    return Reference()
