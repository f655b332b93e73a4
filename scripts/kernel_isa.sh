#!/bin/bash
# Device ISA + resource summary of the slice kernels (code size, VGPRs, SGPRs, scratch).
#   scripts/kernel_isa.sh [tu ...]      (default: every avr_k_*.hip), ISA into /tmp/avr_isa/
cd "$(dirname "$0")/../avrecode_amd"
mkdir -p /tmp/avr_isa
TUS=${@:-avr_k_compress avr_k_decompress avr_k_generate avr_k_seq_compress avr_k_seq_decompress}
for t in $TUS; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S csrc/$t.hip -o /tmp/avr_isa/$t.s 2>/dev/null &
done
wait
for t in $TUS; do
  echo "== $t: $(grep -m1 'codeLenInByte' /tmp/avr_isa/$t.s) $(grep -m1 '; NumVgprs:' /tmp/avr_isa/$t.s) $(grep -m1 '; NumSgprs:' /tmp/avr_isa/$t.s) $(grep -m1 '; ScratchSize:' /tmp/avr_isa/$t.s)"
done
