#!/bin/bash
# TEST INFRASTRUCTURE ONLY: the reference's own extstore.c with the
# INTEGRATION.md section 2 hunks (tests/integration/extstore_ref.patch: the
# batched spill stamp in _submit_wbuf, extstore.c:559, and the open-wbuf read
# fence at extstore.c:886), linked with the driver
# tests/integration/extstore_ref_driver.c and libmcrc32c.so:
#   _ref/extstore_ref           with the fence
#   _ref/extstore_ref_nofence   the fence hunk compiled out (the negative control)
# The reference source is patched in a temporary directory and never copied
# into the repository; extstore.c needs only HAVE_PREAD / HAVE_PREADV from its
# configure-generated config.h (extstore.c:3, :902), given here on the command
# line with an empty config.h beside the copy (as SURVEY.md section 8c compiled
# it).  Run from oracle/ (oracle/Makefile); REF = the reference checkout.
set -e
REF=${REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(dirname "$HERE")
LIB=$ROOT/memcached_amd/libmcrc32c.so
[ -f "$REF/extstore.c" ] || { echo "no $REF/extstore.c: skipped"; exit 0; }
[ -f "$LIB" ] || { echo "build libmcrc32c.so first (python -m memcached_amd.build)"; exit 1; }
T=$(mktemp -d)
trap 'rm -rf "$T"' EXIT
cp "$REF/extstore.c" "$REF/extstore.h" "$T/"
: > "$T/config.h"
patch -s "$T/extstore.c" < "$ROOT/tests/integration/extstore_ref.patch"
mkdir -p "$HERE/_ref"
for v in fence nofence; do
    out=$HERE/_ref/extstore_ref
    def=""
    if [ $v = nofence ]; then out=${out}_nofence; def=-DEXT_NO_FENCE; fi
    ${CC:-gcc} -O2 -Wall -pthread -D_GNU_SOURCE -DHAVE_PREAD -DHAVE_PREADV $def -I"$T" -I"$ROOT/include" \
        "$T/extstore.c" "$ROOT/tests/integration/extstore_ref_driver.c" \
        -L"$ROOT/memcached_amd" -lmcrc32c -Wl,-rpath,'$ORIGIN/../../memcached_amd' -o "$out"
done
