#!/bin/sh
# Build a variant of the lab library (every csrc source, -DCGCK_LAB) for A/B
# runs into con-gen_amd/<name>.so (git-ignored).  Host side only.
#   tools/build_variant.sh NAME FILE 'SED-EXPR'   working tree + one sed edit
#   tools/build_variant.sh NAME --rev REV         the sources of git revision REV
#   tools/build_variant.sh NAME --tree            the working tree as it is (with $VARIANT_FLAGS)
# VARIANT_PRODUCT=1: a product build (no -DCGCK_LAB) instead of a lab one.
set -eu
NAME=$1
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/cgck_variant.XXXXXX)
mkdir -p "$T/con-gen_amd"
if [ "$2" = "--rev" ]; then
	(cd "$R" && git archive "$3" con-gen_amd/csrc include) | tar -x -C "$T"
elif [ "$2" = "--tree" ]; then
	cp -r "$R/con-gen_amd/csrc" "$T/con-gen_amd/csrc"
	ln -s "$R/include" "$T/include"
else
	FILE=$2; EXPR=$3
	cp -r "$R/con-gen_amd/csrc" "$T/con-gen_amd/csrc"
	ln -s "$R/include" "$T/include"   # csrc includes ../../include/cgck.h
	sed -i "$EXPR" "$T/con-gen_amd/csrc/$FILE"
	if cmp -s "$R/con-gen_amd/csrc/$FILE" "$T/con-gen_amd/csrc/$FILE"; then echo "sed changed nothing" >&2; rm -rf "$T"; exit 1; fi
fi
cd "$T/con-gen_amd"
LABFLAG=-DCGCK_LAB=1
[ -n "${VARIANT_PRODUCT:-}" ] && LABFLAG=
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Werror -mcode-object-version=5 \
	-I"$T/include" $LABFLAG ${VARIANT_FLAGS:-} -shared -o "$R/con-gen_amd/$NAME.so" \
	csrc/*.hip csrc/*.cpp
rm -rf "$T"
echo "built con-gen_amd/$NAME.so"
