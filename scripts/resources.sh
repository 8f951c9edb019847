#!/bin/bash
# per-kernel VGPRs / scratch / occupancy of one source (hipcc -Rpass-analysis=kernel-resource-usage)
#   bash scripts/resources.sh render_sphere [extra hipcc flags]
src=$1; shift
flags=""; [ "$src" = render_sphere ] && flags=-fno-slp-vectorize
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Iinclude -Ihyper-ray-tracer_amd/csrc --offload-arch=gfx950 \
  -munsafe-fp-atomics $flags "$@" -c hyper-ray-tracer_amd/csrc/$src.hip -o /tmp/res_$src.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "Function Name|VGPRs:|ScratchSize|Occupancy" | sed -E 's/.*remark: //; s/ \[-Rpass.*//' |
  paste - - - - | awk -F'\t' '{n=$1; sub("Function Name: ","",n); print $2, "|", $3, "|", $4, "|", n}' | c++filt -_ 2>/dev/null | cat
