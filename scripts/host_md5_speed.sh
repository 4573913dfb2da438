#!/bin/bash
# Host per-message MD5: sproxy_amd/csrc/md5_stream.c vs the reference md5.c
# (compiled where it lies), same harness, gcc -O2, messages of 64 B .. 16 KiB.
set -e
cd "$(dirname "$0")/.."
out=build/host_speed; mkdir -p $out
gcc -O2 -o $out/ours tests/c/host_md5_speed.c sproxy_amd/csrc/md5_stream.c -Iinclude
if [ -f /root/reference/md5.c ]; then
  gcc -O2 -include string.h -I/root/reference -o $out/ref tests/c/host_md5_speed.c /root/reference/md5.c
fi
for L in 64 1024 16384; do
  echo "ours $($out/ours $L | tail -1)"
  [ -x $out/ref ] && echo "ref  $($out/ref $L | tail -1)"
done
