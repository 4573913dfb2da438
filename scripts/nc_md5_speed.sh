#!/bin/bash
# Host nc_MD5: sproxy_amd/csrc/nc_md5.c vs the reference
# netcache/netcache/md5.c (compiled where it lies), same harness, gcc -O2,
# cache keys of 32 B .. 1 KiB.  Both give identical digests (tests/test_nc_md5.py).
set -e
cd "$(dirname "$0")/.."
out=build/nc_md5_speed; mkdir -p $out
# build here (sources present); on the GPU box the prebuilt binaries travel in build/
if [ -f sproxy_amd/csrc/nc_md5.c ] && command -v gcc > /dev/null; then
  gcc -O2 -o $out/ours tests/c/nc_md5_speed.c sproxy_amd/csrc/nc_md5.c -Iinclude
fi
if [ -f /root/reference/netcache/netcache/md5.c ]; then
  gcc -O2 -w -I/root/reference/netcache/include -o $out/ref tests/c/nc_md5_speed.c /root/reference/netcache/netcache/md5.c
fi
for L in 32 128 1024; do
  echo "ours $($out/ours $L | tail -1)"
  [ -x $out/ref ] && echo "ref  $($out/ref $L | tail -1)"
done
