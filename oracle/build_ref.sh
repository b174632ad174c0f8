#!/bin/sh
# Builds oracle/_ref/libref_cksum.so from the reference's OWN checksum unit —
# TEST INFRASTRUCTURE ONLY (the referee that pins oracle/cksum_oracle.c).
#
# subr.c as a whole cannot be compiled here: it includes <rte_thash.h>
# unconditionally (subr.c:504) and DPDK is absent, and this recipe writes no
# stand-in for it.  The checksum unit itself, subr.c:119-223 (struct pseudo,
# cksum_add, reduce, cksum_raw, in_cksum, pseudo_cksum, udp_cksum), needs
# nothing but the reference's own subr.h, so that line range is read in place
# from /root/reference and piped straight into the compiler with the
# reference's subr.h force-included.  No reference source is copied to disk;
# only the shared object lands in oracle/_ref/ (git-ignored).
#
# Compile flags follow SConstruct:123-158 (-O2 -DNDEBUG -finline-functions
# -falign-functions=16 -std=gnu99 ...).
set -eu
REF=${CGCK_REFERENCE:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT="$HERE/_ref"
CC=${CC:-gcc}
[ -f "$REF/subr.c" ] || { echo "build_ref: $REF/subr.c absent, skipping"; exit 0; }
first=$(sed -n 119p "$REF/subr.c")
last_fn=$(sed -n 212,213p "$REF/subr.c" | tr -d '\n')
end=$(sed -n 223p "$REF/subr.c")
if [ "$first" != "struct pseudo {" ] || [ "$last_fn" != "uint16_tudp_cksum(struct ip *ip, int len)" ] || [ "$end" != "}" ]; then
	echo "build_ref: subr.c:119-223 is not the checksum unit this recipe expects" >&2
	exit 1
fi
mkdir -p "$OUT"
sed -n 119,223p "$REF/subr.c" | $CC -O2 -DNDEBUG -finline-functions -falign-functions=16 \
	-std=gnu99 -pipe -pthread -fPIC -Wall -Wstrict-prototypes \
	-I"$REF" -include "$REF/subr.h" -x c - -shared -o "$OUT/libref_cksum.so"
echo "build_ref: $OUT/libref_cksum.so"

# The Toeplitz RSS hash: freebsd_rss_key (subr.c:29-35),
# toeplitz_hash (subr.c:482-502) and rss_hash4 (subr.c:506-530), read in place
# the same way.  Line 504, `#include <rte_thash.h>`, sits between the two
# functions and is not part of either, so it is left out of the range.
k0=$(sed -n 29p "$REF/subr.c")
t0=$(sed -n 482,483p "$REF/subr.c" | tr -d '\n')
r0=$(sed -n 506,507p "$REF/subr.c" | cut -c1-9 | tr -d '\n')
r1=$(sed -n 530p "$REF/subr.c")
if [ "$k0" != "uint8_t freebsd_rss_key[RSS_KEY_SIZE] = {" ] || \
   [ "$t0" != "uint32_ttoeplitz_hash(const u_char *data, int cnt, const u_char *key, int key_size)" ] || \
   [ "$r0" != "uint32_trss_hash4" ] || [ "$r1" != "}" ]; then
	echo "build_ref: subr.c:29-35/482-502/506-530 are not the RSS unit this recipe expects" >&2
	exit 1
fi
sed -n '29,35p;482,502p;506,530p' "$REF/subr.c" | $CC -O2 -DNDEBUG -finline-functions -falign-functions=16 \
	-std=gnu99 -pipe -pthread -fPIC -Wall -Wstrict-prototypes \
	-I"$REF" -include "$REF/subr.h" -x c - -shared -o "$OUT/libref_rss.so"
echo "build_ref: $OUT/libref_rss.so"
