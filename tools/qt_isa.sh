#!/bin/bash
# ISA of the production QT kernel (k_substeps_lanes_im<true, true, true>) and its loop's instruction mix
#   bash tools/qt_isa.sh [EXTRA flags]   -> /tmp/qt_im.s + counts
cd "$(dirname "$0")/../mdqtplasmasims_amd/csrc" || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++17 -O3 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function -I/root/repo/include -I/root/repo/mdqtplasmasims_amd/csrc/ -I/opt/rocm/include  -mllvm -amdgpu-sched-strategy=max-ilp $1 --cuda-device-only -S -o /tmp/qtfast.s mdqt_qtfast.hip || exit 1
awk '/^_ZN4mdqt19k_substeps_lanes_imILb1ELb1ELb1EEEvNS_11SubstepArgsEPKNS_7FastTabE:/{f=1} f{print} f&&/s_endpgm/{exit}' /tmp/qtfast.s > /tmp/qt_im.s
grep -E "vgpr_count|sgpr_count|NumVgprs|ScratchSize" /tmp/qtfast.s | grep -A0 -m4 "" > /dev/null
echo "lines $(grep -c '^\s[vsdgb]' /tmp/qt_im.s)  valu $(grep -c '^\s*v_' /tmp/qt_im.s)  salu $(grep -c '^\s*s_' /tmp/qt_im.s)  dpp $(grep -c '_dpp' /tmp/qt_im.s)  nop $(grep -c 's_nop' /tmp/qt_im.s)"
