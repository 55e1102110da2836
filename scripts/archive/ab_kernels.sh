#!/bin/bash
# A/B of the in-tree kernel library against ab/libsn_kernels_old.so on one box:
# tile probe + CaffeNet / GoogLeNet benches, alternating builds.
cd "$GRAFT_REPO_ROOT" || exit 1
OLD=$PWD/ab/libsn_kernels_old.so
for i in 1 2; do
  bash scripts/val.sh old SN_KERNEL_LIB=$OLD -- --steps 100 --warmup 20 || exit 1
  bash scripts/val.sh new -- --steps 100 --warmup 20 || exit 1
done
for i in 1 2; do
  bash scripts/val.sh old-g SN_KERNEL_LIB=$OLD -- --model googlenet --steps 30 --warmup 5 || exit 1
  bash scripts/val.sh new-g -- --model googlenet --steps 30 --warmup 5 || exit 1
done
