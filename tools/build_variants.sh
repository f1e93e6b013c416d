#!/bin/bash
# Builds experiment variants of the library: exp/lib<name>.so with -D<macros>.  Usage: build_variants.sh name:MACRO,MACRO ...
set -eu
mkdir -p exp
cd gossip-protocol_amd
SRCS=$(sed -n 's/^SRCS *:= *//p' Makefile)
for spec in "$@"; do
  name=${spec%%:*}; macros=${spec#*:}; defs=""
  for m in ${macros//,/ }; do [ -n "$m" ] && [ "$m" != "$name" ] && defs="$defs -D$m"; done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-result $defs \
    $SRCS -o ../exp/lib$name.so &
done
wait
