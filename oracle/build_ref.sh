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
