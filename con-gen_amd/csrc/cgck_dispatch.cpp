// cgck_dispatch.cpp — picks the kernel family and launch shape for a batch.
//
// The product library (libcgck.so) carries only the families the dispatcher
// picks by itself: dstr (dense strided >= 1 KiB frames, the 1500 B config),
// group (>= 1 KiB typical length otherwise, drop-in and window calls),
// lpd / lpa (aligned fixed-length 20..64-byte strided batches), lpp (small
// unaligned or descriptor packets) and slot2 (mid-size / mixed lengths).  The
// A/B-only variants measured against them (slot, lppp, the other lpp shapes,
// the LDS-DMA stream kernels, the probe kernels) are compiled only into
// libcgck_lab.so (-DCGCK_LAB, tools/Makefile) for tools/ab_inproc.py and
// tools/sweep.py.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>

#include "cgck_internal.h"

namespace cgck {

thread_local const char *t_kernel = "";

const char *intern(const char *fmt, ...)
{
	// called once per launch site (function-local static): the strings live
	// for the process
	static std::mutex mu;
	char buf[128];
	va_list ap;
	va_start(ap, fmt);
	vsnprintf(buf, sizeof(buf), fmt, ap);
	va_end(ap);
	std::lock_guard<std::mutex> lk(mu);
	return strdup(buf);
}

hipError_t launch_group(const KParams &p, uint32_t max_len, int num_cus, bool nt, hipStream_t st);
hipError_t launch_lpp(const KParams &p, int num_cus, bool nt, int shape, hipStream_t st);
hipError_t launch_slot2(const KParams &p, int num_cus, bool nt, hipStream_t st);
hipError_t launch_lpa(const KParams &p, int num_cus, bool nt, hipStream_t st);
hipError_t launch_lpd(const KParams &p, int num_cus, hipStream_t st);
bool lpd_ok(const KParams &p);
hipError_t launch_lpw(const KParams &p, int num_cus, hipStream_t st);
bool lpw_ok(const KParams &p);
hipError_t launch_dstr(const KParams &p, int num_cus, hipStream_t st);
bool dstr_ok(const KParams &p);
#if CGCK_LAB
hipError_t launch_span(const KParams &p, int num_cus, bool nt, hipStream_t st);
bool span_ok(const KParams &p);
hipError_t launch_slot(const KParams &p, int num_cus, bool nt, hipStream_t st);
hipError_t launch_lppp(const KParams &p, int num_cus, bool nt, hipStream_t st);
hipError_t launch_stream(const KParams &p, int num_cus, hipStream_t st);
bool stream_ok(const KParams &p);
hipError_t launch_slotd(const KParams &p, int num_cus, hipStream_t st);
#endif

// `kernel` = variant | flags (cgck_ctx_set_kernel pins the variant by family
// name; in the lab build so does $CGCK_KERNEL):
//   variant (bits 0-3): 0 auto, 1 group (G lanes per packet), 2 lane per
//     packet (lpp), 9 lane per 128-byte slot pipelined two deep (slot2, the
//     default for mid-size packets), 10 lane per packet for aligned
//     fixed-length strided 20..64-byte packets, A/B pipelined (lpa), 13 the
//     same fed by LDS-DMA with staged output runs (lpd, the default there when
//     the batch has no verdicts, counters or stores and stride <= 64), 15
//     lane per packet over DMA'd windows of a packed step's span (lpw, the
//     default for descriptor batches of mixed lengths below 1 KiB under
//     cgck_set_desc_layout(PACKED)), 11 dense strided frames streamed through
//     LDS by DMA, four per step, with a writer wave (dstr, cgck_dense.hip: the
//     default for strided batches of >= 1 KiB frames it accepts, dstr_ok;
//     $CGCK_STR_OLD in the lab build: the first stream kernel,
//     cgck_stream.hip).  libcgck_lab.so only: 3 lane per 128-byte
//     slot, 4 software-pipelined lane per packet, 5..8 lpp shapes 1..3, 0,
//     12 the packed span (coalesced
//     register stream + prefix sums, cgck_span.hip), 14 lane per slot fed by
//     LDS-DMA (slotd).  A variant this build lacks falls back to the automatic
//     choice; one whose preconditions a batch fails falls back to lpa, lpp or
//     group;
//   kNT (bit 4) nontemporal loads, kContig (bit 5) contiguous block ranges,
//   kExplicit (bit 6) take bits 4-5 as given instead of the measured defaults,
//   kPacked (bit 7) the context's layout hint says packed (cgck_set_desc_layout).
// len_hint = the batch's packet length (strided) or typical length (descriptors).
hipError_t launch_cksum(const KParams &p0, uint32_t len_hint, int num_cus, int kernel, hipStream_t st)
{
	if (p0.n == 0)
		return hipSuccess;
	KParams p = p0;
	const bool lane_ok = !(p.flags & (kFlagNoLenCheck | kFlagL4Auto | kFlagRx | kFlagGroup));
	int variant = kernel & 15;
	// aligned fixed-length strided batch of 20..64-byte packets (the 64 B config)
	const bool lpa_ok = lane_ok && !p.desc && p.ip_len >= 20 && p.ip_len <= 64 &&
			    ((reinterpret_cast<uintptr_t>(p.base) | p.stride | p.l3_off) & 15) == 0;
#if CGCK_LAB
	const bool known = variant <= 15;
#else
	const bool known = variant == 1 || variant == 2 || variant == 9 || variant == 10 || variant == 11 ||
			   variant == 13 || variant == 15;
#endif
	// 256 B <= typical length < 1 KiB: lpw streams 64-frame steps through LDS
	// by DMA, the step's span itself when its frames lie back to back and the
	// frames' chunk runs gathered otherwise, decided per step on the device
	// (tools/family_ab.py, profiles/r03/: 16M IMIX packed without a hint 73.0 %
	// vs slot2 62.8 %, in 2048 B ring slots at +14 62.0 vs 45.7 %; dense strided
	// 256 / 576 / 1000 B 69.6 / 73.1 / 74.7 % vs slot2's 52.1 / 56.6 / 48.4 %,
	// profiles/r02/dma/lpw; 160 B 46.9 vs 59.8 %, 1500 B 75.6 vs group 79.9 %).
	// The layout hint (kPacked) no longer changes the choice.
	const bool stream = len_hint >= kLpwFromLen && lpw_ok(p) && (p.desc || p.stride > 0);
	if (variant == 0 || !known)
		variant = !lane_ok ? 1 : lpa_ok ? (lpd_ok(p) ? 13 : 10)
			: len_hint >= kGroupFromLen ? (!p.desc && dstr_ok(p) ? 11 : 1)
			: len_hint <= kLppUpToLen ? 2 : stream ? 15 : 9;
	if (variant >= 2 && !lane_ok)
		variant = 1;
	if (variant == 10 && !lpa_ok)
		variant = 2;
	if (variant == 13 && !(lpa_ok && lpd_ok(p)))
		variant = lpa_ok ? 10 : 2;
#if CGCK_LAB
	if (variant == 12 && !span_ok(p))
		variant = 1;
#endif
	if (variant == 11 && !dstr_ok(p))
		variant = 1;
	if (variant == 15 && !lpw_ok(p))
		variant = lane_ok ? 9 : 1;
	bool nt, contig;
	if (kernel & kExplicit) {
		nt = kernel & kNT;
		contig = kernel & kContig;
	} else if (variant == 1) {
		nt = kDefaultGroupNT;
		contig = kDefaultGroupContig;
	} else {
		nt = kDefaultLaneNT;
		contig = kDefaultLaneContig;
	}
	p.contig = contig;
	switch (variant) {
	case 2:
		return launch_lpp(p, num_cus, nt, kDefaultLppShape, st);
	case 9:
		return launch_slot2(p, num_cus, nt, st);
	case 10:
		return launch_lpa(p, num_cus, nt, st);
	case 13:
		return launch_lpd(p, num_cus, st);
	case 15:
		return launch_lpw(p, num_cus, st);
	case 11:
#if CGCK_LAB
		if (CGCK_ENV("CGCK_STR_OLD") && stream_ok(p)) // the first stream kernel (cgck_stream.hip)
			return launch_stream(p, num_cus, st);
#endif
		return launch_dstr(p, num_cus, st);
#if CGCK_LAB
	case 12:
		return launch_span(p, num_cus, nt, st);
	case 3:
		return launch_slot(p, num_cus, nt, st);
	case 4:
		return launch_lppp(p, num_cus, nt, st);
	case 5:
		return launch_lpp(p, num_cus, nt, 1, st);
	case 6:
		return launch_lpp(p, num_cus, nt, 2, st);
	case 7:
		return launch_lpp(p, num_cus, nt, 3, st);
	case 8:
		return launch_lpp(p, num_cus, nt, 0, st);
	case 14:
		return launch_slotd(p, num_cus, st);
#endif
	default:
		return launch_group(p, len_hint, num_cus, nt, st);
	}
}

} // namespace cgck
