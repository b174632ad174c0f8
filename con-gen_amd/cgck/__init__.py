"""cgck — Python binding of libcgck.so, the gfx950 Internet-checksum engine.

Mirrors the reference's checksum interface (subr.h:176-177, 373-374):

    in_cksum(buf, off, n)        uint16_t in_cksum(void *, int)
    udp_cksum(buf, ip_off, n)    uint16_t udp_cksum(struct ip *, int)
    ip_cksum(buf, ip_off)        #define ip_cksum(ip) in_cksum(ip, ip->ip_hl << 2)
    tcp_cksum                    #define tcp_cksum udp_cksum

plus the batched C-ABI of include/cgck.h (`Engine`).  Everything here calls
the HIP kernels through the C-ABI; there is no Python or host arithmetic
path, and loading fails loudly when the library is missing.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CGCK_LIB", os.path.join(os.path.dirname(HERE), "libcgck.so"))

# Flags and verdict bits (include/cgck.h).
RAW = 1 << 0
IP = 1 << 1
L4 = 1 << 2
L4_NOPSEUDO = 1 << 3
ZERO_FIELDS = 1 << 4
STORE = 1 << 5
VERIFY = 1 << 6
V_IP_ZERO_IS_FFFF = 1 << 7
V_UDP_ZERO_SKIP = 1 << 8
GEN_BOTH = IP | L4
FILL_BOTH = IP | L4 | ZERO_FIELDS | STORE
VERIFY_BSD = IP | L4 | VERIFY | V_IP_ZERO_IS_FFFF | V_UDP_ZERO_SKIP
VERIFY_TOY = IP | L4 | VERIFY
BAD_IP = 1
BAD_L4 = 2
BAD_LEN = 4

# cgck_dst_entry_t (include/cgck.h): the struct ip_socket fields con-gen.c:344-349 fills.
DST_DTYPE = np.dtype([("laddr", "<u4"), ("faddr", "<u4"), ("lport", "<u2"), ("fport", "<u2"),
                      ("hash", "<u4")])
assert DST_DTYPE.itemsize == 16


class DstParams(ctypes.Structure):
    """cgck_dst_params_t: the struct thread fields thread_init_dst_cache reads."""
    _fields_ = [("laddr_min", ctypes.c_uint32), ("laddr_max", ctypes.c_uint32),
                ("faddr_min", ctypes.c_uint32), ("faddr_max", ctypes.c_uint32),
                ("fport", ctypes.c_uint16), ("rss_queue_num", ctypes.c_uint8),
                ("rss_queue_id", ctypes.c_uint8), ("rss_key", ctypes.c_void_p),
                ("rss_key_size", ctypes.c_int)]


DESC_DTYPE = np.dtype([("frame_off", "<u8"), ("l3_off", "<u2"), ("ip_len", "<u2")], align=False)
assert DESC_DTYPE.itemsize == 12

# Every symbol include/cgck.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "in_cksum", "udp_cksum", "cgck_last_error", "cgck_abi_version", "cgck_ctx_create",
    "cgck_ctx_destroy", "cgck_ctx_stream", "cgck_ctx_sync", "cgck_strided", "cgck_desc",
    "cgck_set_desc_len_hint", "cgck_desc_host", "cgck_host_register", "cgck_host_unregister",
    "cgck_thread_release", "cgck_tx_begin", "cgck_tx_flush", "cgck_synth_strided",
    "cgck_synth_imix", "cgck_imix_bytes", "cgck_device_count", "cgck_dev_alloc", "cgck_dev_free",
    "cgck_host_alloc", "cgck_host_free", "cgck_memcpy", "cgck_memset", "cgck_event_create",
    "cgck_event_destroy", "cgck_event_record", "cgck_event_elapsed_ms", "cgck_probe_read",
    "toeplitz_hash", "rss_hash4", "cgck_toeplitz", "cgck_dst_cache", "cgck_dst_cache_host",
    "cgck_burst_open", "cgck_burst_close", "cgck_thread_ctx", "cgck_set_error_handler",
    "cgck_rx_begin", "cgck_rx_end", "cgck_window_stats", "cgck_ctx_last_kernel", "cgck_set_desc_layout",
    "cgck_ctx_set_kernel", "cgck_synth_imix_ring", "cgck_burst_request", "cgck_host_device_ptr",
    "cgck_rx_post", "cgck_rx_begin_posted", "cgck_tx_post", "cgck_tx_complete",
    "cgck_rx_pending", "cgck_rx_ready", "cgck_tx_pending", "cgck_tx_ready",
    "cgck_window_stats_n", "cgck_thread_bind", "cgck_thread_device",
    "cgck_test_burst_seq", "cgck_test_burst_stale",
)
# Descriptor layout hint (cgck_set_desc_layout)
LAYOUT_ANY = 0
LAYOUT_PACKED = 1
LAB_PATH = os.path.join(os.path.dirname(HERE), "libcgck_lab.so")

# cgck_error_fn: void (*)(const char *what, const char *msg, void *arg)
ERROR_FN = ctypes.CFUNCTYPE(None, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p)


class CgckError(RuntimeError):
    pass


_lib = None
_vp = ctypes.c_void_p
_u64 = ctypes.c_uint64
_u32 = ctypes.c_uint32


def load(path=None):
    """Load libcgck.so (once).  Raises if it is missing: there is no fallback."""
    global _lib
    if _lib is None:
        _lib = bind(path or LIB_PATH)
    return _lib


def bind(path):
    """A ctypes binding of one libcgck.so build (tools/ab_inproc.py loads two
    builds into one process this way; everything else goes through load())."""
    if not os.path.exists(path):
        raise CgckError(f"libcgck.so not built at {path} (run make -C con-gen_amd)")
    L = ctypes.CDLL(path)
    L.in_cksum.restype = ctypes.c_uint16
    L.in_cksum.argtypes = [_vp, ctypes.c_int]
    L.udp_cksum.restype = ctypes.c_uint16
    L.udp_cksum.argtypes = [_vp, ctypes.c_int]
    L.cgck_last_error.restype = ctypes.c_char_p
    L.cgck_abi_version.restype = ctypes.c_int
    L.cgck_device_count.restype = ctypes.c_int
    L.cgck_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(_vp)]
    L.cgck_ctx_destroy.argtypes = [_vp]
    L.cgck_ctx_stream.restype = _vp
    L.cgck_ctx_stream.argtypes = [_vp]
    L.cgck_ctx_sync.argtypes = [_vp]
    L.cgck_ctx_set_kernel.argtypes = [_vp, ctypes.c_char_p]
    L.cgck_set_desc_len_hint.argtypes = [_vp, _u32]
    L.cgck_set_desc_layout.argtypes = [_vp, _u32]
    L.cgck_strided.argtypes = [_vp, _vp, _u64, _u64, _u32, _u32, _u32, _vp, _vp, _vp, _vp]
    L.cgck_desc.argtypes = [_vp, _vp, _vp, _u64, _u32, _vp, _vp, _vp, _vp]
    L.cgck_desc_host.argtypes = [_vp, _vp, ctypes.c_size_t, _vp, _u64, _u32, _vp, _vp]
    L.cgck_host_register.argtypes = [_vp, ctypes.c_size_t]
    L.cgck_host_unregister.argtypes = [_vp]
    L.cgck_synth_strided.argtypes = [_vp, _vp, _u64, _u64, _u32, _u64, _vp]
    L.cgck_synth_imix.argtypes = [_vp, _vp, _vp, _u64, _u64, _vp]
    L.cgck_synth_imix_ring.argtypes = [_vp, _vp, _vp, _u64, _u64, _u32, _u64, _vp]
    L.cgck_imix_bytes.restype = _u64
    L.cgck_imix_bytes.argtypes = [_u64]
    L.cgck_dev_alloc.argtypes = [ctypes.c_size_t, ctypes.POINTER(_vp)]
    L.cgck_dev_free.argtypes = [_vp]
    L.cgck_host_alloc.argtypes = [ctypes.c_size_t, ctypes.POINTER(_vp)]
    L.cgck_host_free.argtypes = [_vp]
    L.cgck_memcpy.argtypes = [_vp, _vp, ctypes.c_size_t, _vp]
    L.cgck_memset.argtypes = [_vp, ctypes.c_int, ctypes.c_size_t, _vp]
    L.cgck_event_create.argtypes = [ctypes.POINTER(_vp)]
    L.cgck_event_destroy.argtypes = [_vp]
    L.cgck_event_record.argtypes = [_vp, _vp, _vp]
    L.cgck_event_elapsed_ms.argtypes = [_vp, _vp, ctypes.POINTER(ctypes.c_float)]
    L.cgck_probe_read.argtypes = [_vp, _vp, _u64, _vp, _vp]
    L.toeplitz_hash.restype = _u32
    L.toeplitz_hash.argtypes = [_vp, ctypes.c_int, _vp, ctypes.c_int]
    L.rss_hash4.restype = _u32
    L.rss_hash4.argtypes = [_u32, _u32, ctypes.c_uint16, ctypes.c_uint16, _vp, ctypes.c_int]
    L.cgck_toeplitz.argtypes = [_vp, _vp, _u64, _u64, _u32, _vp, ctypes.c_int, _u32, _vp, _vp]
    L.cgck_dst_cache.argtypes = [_vp, ctypes.POINTER(DstParams), _vp, _u32, _vp, _vp]
    L.cgck_dst_cache_host.argtypes = [_vp, ctypes.POINTER(DstParams), _vp, _u32,
                                      ctypes.POINTER(_u32)]
    L.cgck_burst_open.argtypes = [_vp, _u32, ctypes.c_size_t, _u32]
    L.cgck_burst_close.argtypes = [_vp]
    if hasattr(L, "cgck_burst_request"):   # ABI additions of round 4 (an older build loads without them)
        L.cgck_burst_request.argtypes = [_vp, _vp, _u64, _vp, _u64, _u32, _vp, _vp]
        L.cgck_host_device_ptr.argtypes = [_vp, ctypes.c_size_t, ctypes.POINTER(_vp)]
    L.cgck_thread_ctx.restype = _vp
    L.cgck_set_error_handler.restype = None
    L.cgck_set_error_handler.argtypes = [ERROR_FN, _vp]
    L.cgck_rx_begin.argtypes = [_vp, ctypes.c_size_t, _vp, _u64]
    if hasattr(L, "cgck_rx_post"):
        L.cgck_rx_post.argtypes = [_vp, ctypes.c_size_t, _vp, _u64]
    L.cgck_window_stats.argtypes = [ctypes.POINTER(_u64)]
    if hasattr(L, "cgck_window_stats_n"):   # ABI additions of round 6
        L.cgck_window_stats_n.argtypes = [ctypes.POINTER(_u64), ctypes.c_int]
        L.cgck_thread_bind.argtypes = [ctypes.c_int]
    L.cgck_ctx_last_kernel.restype = ctypes.c_char_p
    L.cgck_ctx_last_kernel.argtypes = [_vp]
    return L


def _check(rc, what):
    if rc < 0:
        msg = _lib.cgck_last_error().decode(errors="replace")
        raise CgckError(f"{what} failed ({rc}): {msg}")
    return rc


def device_count():
    return load().cgck_device_count()


# ---------------------------------------------------------------------------
# Drop-in interface (reference names and argument meaning).
# ---------------------------------------------------------------------------

def _addr(buf, off):
    if not isinstance(buf, np.ndarray) or buf.dtype != np.uint8:
        raise TypeError("buf must be a numpy uint8 array")
    return buf.ctypes.data + off


def in_cksum(buf, off=0, n=None):
    """in_cksum(buf + off, n) — subr.c:186-195, on the GPU."""
    if n is None:
        n = len(buf) - off
    return load().in_cksum(_addr(buf, off), n)


def udp_cksum(buf, ip_off, n):
    """udp_cksum((struct ip *)(buf + ip_off), n) — subr.c:212-223, on the GPU."""
    return load().udp_cksum(_addr(buf, ip_off), n)


tcp_cksum = udp_cksum


def ip_cksum(buf, ip_off=0):
    """ip_cksum(ip) = in_cksum(ip, ip->ip_hl << 2) — subr.h:176."""
    return in_cksum(buf, ip_off, (int(buf[ip_off]) & 0x0F) << 2)


def _u8(a):
    return np.ascontiguousarray(np.frombuffer(bytes(a), np.uint8) if isinstance(a, (bytes, bytearray))
                                else a, np.uint8)


def toeplitz_hash(data, key, cnt=None, key_size=None):
    """toeplitz_hash(data, cnt, key, key_size) — subr.c:482-502, on the GPU."""
    d, k = _u8(data), _u8(key)
    return load().toeplitz_hash(d.ctypes.data, len(d) if cnt is None else cnt, k.ctypes.data,
                                len(k) if key_size is None else key_size)


def rss_hash4(laddr, faddr, lport, fport, key, key_size=None):
    """rss_hash4(laddr, faddr, lport, fport, key, key_size) — subr.c:506-530
    (arguments in network order, as con-gen.c:338 passes them), on the GPU."""
    k = _u8(key)
    return load().rss_hash4(laddr, faddr, lport, fport, k.ctypes.data,
                            len(k) if key_size is None else key_size)


def burst_open(max_pkts=4096, max_bytes=4 << 20, idle_ms=0):
    """cgck_burst_open(NULL, ...): the resident burst server on this thread's
    drop-in context."""
    _check(load().cgck_burst_open(None, max_pkts, max_bytes, idle_ms), "cgck_burst_open")


def burst_close():
    _check(load().cgck_burst_close(None), "cgck_burst_close")


def last_error():
    """cgck_last_error(): this thread's last error text."""
    return load().cgck_last_error().decode()


def host_device_ptr(arr, nbytes=None):
    """cgck_host_device_ptr: the device view of a registered numpy buffer."""
    p = _vp()
    _check(load().cgck_host_device_ptr(arr.ctypes.data, arr.nbytes if nbytes is None else nbytes,
                                       ctypes.byref(p)), "cgck_host_device_ptr")
    return p.value


def fn_pointers():
    """(in_cksum, udp_cksum) addresses in libcgck.so, for C harnesses that
    call the drop-in symbols (oracle.Port.replay_rx, oracle_cpu_bench)."""
    L = load()
    return (ctypes.cast(L.in_cksum, ctypes.c_void_p).value,
            ctypes.cast(L.udp_cksum, ctypes.c_void_p).value)


def rx_begin(base, desc):
    """cgck_rx_begin over a numpy byte array (the ring) and DESC_DTYPE
    descriptors (ip_len = bytes received after l3_off).  Returns the number
    of frames precomputed."""
    assert desc.dtype == DESC_DTYPE
    return _check(load().cgck_rx_begin(base.ctypes.data, base.nbytes, desc.ctypes.data, len(desc)),
                  "cgck_rx_begin")


def rx_end():
    """cgck_rx_end: returns how many drop-in calls the window answered."""
    return _check(load().cgck_rx_end(), "cgck_rx_end")


def rx_post(base, desc):
    """cgck_rx_post: post a burst (numpy ring + descriptors); returns the
    frames posted.  The ring and the descriptors' frames must stay unchanged
    until its window (rx_begin_posted .. rx_end) closes."""
    assert desc.dtype == DESC_DTYPE
    return _check(load().cgck_rx_post(base.ctypes.data, base.nbytes, desc.ctypes.data, len(desc)),
                  "cgck_rx_post")


def rx_begin_posted():
    """cgck_rx_begin_posted: open the window over the oldest posted burst."""
    return _check(load().cgck_rx_begin_posted(), "cgck_rx_begin_posted")


def rx_pending():
    """cgck_rx_pending: bursts posted and not yet opened (the drain rule)."""
    return _check(load().cgck_rx_pending(), "cgck_rx_pending")


def rx_ready():
    """cgck_rx_ready: 1 when the oldest posted burst's values are in, 0 while
    the GPU still computes it (no wait)."""
    return _check(load().cgck_rx_ready(), "cgck_rx_ready")


def tx_pending():
    """cgck_tx_pending: fills posted and not yet completed."""
    return _check(load().cgck_tx_pending(), "cgck_tx_pending")


def tx_ready():
    """cgck_tx_ready: 1 when the oldest posted fill's values are in (no wait)."""
    return _check(load().cgck_tx_ready(), "cgck_tx_ready")


def window_stats():
    """[rx served, rx synchronous, tx queued, tx synchronous] of this thread."""
    a = (_u64 * 4)()
    _check(load().cgck_window_stats(a), "cgck_window_stats")
    return list(a)


def window_stats_n():
    """window_stats() plus [4]: TX-window calls queued on a header of the
    last closed RX window's frames (cgck_window_stats_n)."""
    a = (_u64 * 8)()
    k = _check(load().cgck_window_stats_n(a, 8), "cgck_window_stats_n")
    return list(a)[:k]


def thread_bind(device):
    """cgck_thread_bind: this thread's drop-in context goes on `device`."""
    return _check(load().cgck_thread_bind(device), "cgck_thread_bind")


def thread_device():
    return load().cgck_thread_device()


_err_cb = None


def set_error_handler(fn):
    """cgck_set_error_handler: fn(what: str, msg: str) (None restores the
    default).  The drop-ins abort if the handler returns."""
    global _err_cb
    _err_cb = None if fn is None else ERROR_FN(lambda w, m, a: fn(w.decode(), m.decode()))
    load().cgck_set_error_handler(_err_cb if _err_cb is not None else ERROR_FN(), None)


def tx_begin():
    _check(load().cgck_tx_begin(), "cgck_tx_begin")


def tx_flush():
    return _check(load().cgck_tx_flush(), "cgck_tx_flush")


def tx_post():
    """cgck_tx_post: post the window's fill; returns the fields queued."""
    return _check(load().cgck_tx_post(), "cgck_tx_post")


def tx_complete():
    """cgck_tx_complete: wait for the oldest posted fill and write its fields."""
    return _check(load().cgck_tx_complete(), "cgck_tx_complete")


def thread_release():
    load().cgck_thread_release()


# ---------------------------------------------------------------------------
# Batched engine (device memory owned by the library).
# ---------------------------------------------------------------------------

class DeviceBuffer:
    def __init__(self, nbytes):
        L = load()
        p = _vp()
        _check(L.cgck_dev_alloc(nbytes, ctypes.byref(p)), "cgck_dev_alloc")
        self.ptr = p.value
        self.nbytes = nbytes

    def free(self):
        if self.ptr:
            load().cgck_dev_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def upload(self, arr, off=0, stream=None):
        arr = np.ascontiguousarray(arr)
        assert off + arr.nbytes <= self.nbytes
        _check(load().cgck_memcpy(self.ptr + off, arr.ctypes.data, arr.nbytes, stream), "upload")

    def download(self, arr, off=0, stream=None):
        assert arr.flags.c_contiguous and off + arr.nbytes <= self.nbytes
        _check(load().cgck_memcpy(arr.ctypes.data, self.ptr + off, arr.nbytes, stream), "download")


class Event:
    def __init__(self):
        p = _vp()
        _check(load().cgck_event_create(ctypes.byref(p)), "cgck_event_create")
        self.ptr = p.value

    def __del__(self):
        try:
            load().cgck_event_destroy(self.ptr)
        except Exception:
            pass


class Engine:
    """One context (stream + staging) on one device — use one per thread."""

    def __init__(self, device=0, kernel=None):
        L = load()
        p = _vp()
        _check(L.cgck_ctx_create(device, ctypes.byref(p)), "cgck_ctx_create")
        self.ctx = p.value
        self.device = device
        if kernel is not None:
            self.set_kernel(kernel)

    def set_kernel(self, family):
        """cgck_ctx_set_kernel: pin the kernel family ("auto", "group", "lpp",
        "lpa", "slot2", "dstr", "lpd", "lpw"; the lab build knows more)."""
        _check(load().cgck_ctx_set_kernel(self.ctx, family.encode()), "cgck_ctx_set_kernel")

    def close(self):
        if self.ctx:
            load().cgck_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self):
        return load().cgck_ctx_stream(self.ctx)

    @property
    def last_kernel(self):
        """The kernel the dispatcher launched last on this context (the name
        rocprofv3 reports)."""
        return load().cgck_ctx_last_kernel(self.ctx).decode()

    def sync(self):
        _check(load().cgck_ctx_sync(self.ctx), "cgck_ctx_sync")

    def burst_open(self, max_pkts=4096, max_bytes=4 << 20, idle_ms=0):
        """cgck_burst_open: keep a burst server resident on this context."""
        _check(load().cgck_burst_open(self.ctx, max_pkts, max_bytes, idle_ms), "cgck_burst_open")

    def burst_close(self):
        _check(load().cgck_burst_close(self.ctx), "cgck_burst_close")

    def burst_request(self, dev_base, range_bytes, desc, flags, out=None, verdict=None):
        """cgck_burst_request: one request to the open server over device-visible
        memory [dev_base, +range_bytes); the server checks the descriptors.
        Returns the library's return code (0, -EIO refused, -ENOSPC)."""
        assert desc.dtype == DESC_DTYPE
        return load().cgck_burst_request(self.ctx, dev_base, range_bytes, desc.ctypes.data, len(desc), flags,
                                         None if out is None else out.ctypes.data,
                                         None if verdict is None else verdict.ctypes.data)

    def set_desc_len_hint(self, n):
        _check(load().cgck_set_desc_len_hint(self.ctx, n), "cgck_set_desc_len_hint")

    def set_desc_layout(self, layout):
        """cgck_set_desc_layout: LAYOUT_PACKED for descriptor batches whose
        frames lie back to back (picks the streaming kernel, lpw)."""
        _check(load().cgck_set_desc_layout(self.ctx, layout), "cgck_set_desc_layout")

    def strided(self, base, n, stride, l3_off, ip_len, flags, out=None, verdict=None, bad=None,
                stream=None):
        """Device pointers in, asynchronous (cgck_strided)."""
        _check(load().cgck_strided(self.ctx, base, n, stride, l3_off, ip_len, flags, out, verdict,
                                   bad, stream), "cgck_strided")

    def desc(self, base, desc, n, flags, out=None, verdict=None, bad=None, stream=None):
        _check(load().cgck_desc(self.ctx, base, desc, n, flags, out, verdict, bad, stream),
               "cgck_desc")

    def desc_host(self, base, desc, flags, out=None, verdict=None):
        """Host-resident batch (numpy): H2D, kernel, D2H.  Synchronous."""
        n = len(desc)
        assert desc.dtype == DESC_DTYPE
        _check(load().cgck_desc_host(self.ctx, base.ctypes.data, base.nbytes, desc.ctypes.data, n,
                                     flags, None if out is None else out.ctypes.data,
                                     None if verdict is None else verdict.ctypes.data),
               "cgck_desc_host")

    def synth_strided(self, base, n, stride, ip_len, seed, stream=None):
        _check(load().cgck_synth_strided(self.ctx, base, n, stride, ip_len, seed, stream),
               "cgck_synth_strided")

    def synth_imix(self, base, desc, n, seed, stream=None):
        _check(load().cgck_synth_imix(self.ctx, base, desc, n, seed, stream), "cgck_synth_imix")

    def synth_imix_ring(self, base, desc, n, stride, l3_off, seed, stream=None):
        """IMIX frames in ring slots (cgck_synth_imix_ring): n * stride bytes at base."""
        _check(load().cgck_synth_imix_ring(self.ctx, base, desc, n, stride, l3_off, seed, stream),
               "cgck_synth_imix_ring")

    def toeplitz(self, data, n, stride, cnt, key, out, mask=0xFFFFFFFF, key_size=None, stream=None):
        """cgck_toeplitz: device data/out, host key.  Asynchronous."""
        k = _u8(key)
        _check(load().cgck_toeplitz(self.ctx, data, n, stride, cnt, k.ctypes.data,
                                    len(k) if key_size is None else key_size, mask, out, stream),
               "cgck_toeplitz")

    @staticmethod
    def dst_params(laddr, faddr, fport, queue_num, queue_id, key=None, key_size=None):
        """laddr/faddr = (min, max) host order; fport network order.  The key
        array must stay alive while the params are used."""
        k = None if key is None else _u8(key)
        p = DstParams(laddr[0], laddr[1], faddr[0], faddr[1], fport, queue_num, queue_id,
                      None if k is None else k.ctypes.data,
                      0 if k is None else (len(k) if key_size is None else key_size))
        p._key_ref = k
        return p

    def dst_cache(self, params, out, cap, count, stream=None):
        """cgck_dst_cache: device out/count, asynchronous."""
        _check(load().cgck_dst_cache(self.ctx, ctypes.byref(params), out, cap, count, stream),
               "cgck_dst_cache")

    def dst_cache_host(self, params, cap):
        """cgck_dst_cache_host: returns the DST_DTYPE entries written."""
        out = np.zeros(cap, DST_DTYPE)
        got = _u32()
        _check(load().cgck_dst_cache_host(self.ctx, ctypes.byref(params), out.ctypes.data, cap,
                                          ctypes.byref(got)), "cgck_dst_cache_host")
        return out[:got.value]

    def probe_read(self, src, nbytes, sink, stream=None):
        _check(load().cgck_probe_read(self.ctx, src, nbytes, sink, stream), "cgck_probe_read")

    def record(self, ev, stream=None):
        _check(load().cgck_event_record(self.ctx, ev.ptr, stream), "cgck_event_record")

    @staticmethod
    def elapsed_ms(a, b):
        ms = ctypes.c_float()
        _check(load().cgck_event_elapsed_ms(a.ptr, b.ptr, ctypes.byref(ms)), "elapsed")
        return ms.value

    # -- numpy conveniences (tests) --
    def run_host_strided(self, buf, n, stride, l3_off, ip_len, flags, want_verdict=True):
        """Copy a host batch to the device, run cgck_strided, copy results (and,
        with STORE, the bytes) back.  Returns (out, verdict); verdict is None
        when want_verdict is False (no verdict array passed to the library)."""
        d = DeviceBuffer(max(buf.nbytes, 1))
        o = DeviceBuffer(4 * max(n, 1))
        v = DeviceBuffer(max(n, 1))
        d.upload(buf, stream=self.stream)
        self.strided(d.ptr, n, stride, l3_off, ip_len, flags, o.ptr, v.ptr if want_verdict else None, None)
        out = np.zeros(n, np.uint32)
        ver = np.zeros(n, np.uint8) if want_verdict else None
        o.download(out, stream=self.stream)
        if want_verdict:
            v.download(ver, stream=self.stream)
        if flags & STORE:
            d.download(buf, stream=self.stream)
        self.sync()
        return out, ver

    def run_host_desc(self, buf, desc, flags):
        n = len(desc)
        d = DeviceBuffer(max(buf.nbytes, 1))
        dd = DeviceBuffer(max(desc.nbytes, 12))
        o = DeviceBuffer(4 * max(n, 1))
        v = DeviceBuffer(max(n, 1))
        d.upload(buf, stream=self.stream)
        dd.upload(desc, stream=self.stream)
        self.desc(d.ptr, dd.ptr, n, flags, o.ptr, v.ptr, None)
        out = np.zeros(n, np.uint32)
        ver = np.zeros(n, np.uint8)
        o.download(out, stream=self.stream)
        v.download(ver, stream=self.stream)
        if flags & STORE:
            d.download(buf, stream=self.stream)
        self.sync()
        return out, ver
