# ISA inspection of scan_kernel<false,false,0> (K= another mangled name) for compile-time variants (CPU only):
#   bash tools/isa_check.sh "" "-DSOME_EXPERIMENT=1" ...
K=${K:-_ZN3srd11scan_kernelILb0ELb0ELi0EEEvNS_8ScanArgsE}  # scan_kernel<false,false,0>
# Prints VGPRs, scratch, and the vmcnt waits / loads of the main ring loop.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/isa_check
mkdir -p $W
for v in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 $v -I$R/include -I$R/rust-simd-r-drive_amd/csrc \
    --cuda-device-only -S -o $W/t.s $R/rust-simd-r-drive_amd/csrc/srd_api.hip 2>&1 | grep -i " error" || true
  a=$(grep -n "^$K:" $W/t.s | cut -d: -f1)
  b=$(grep -n "^.Lfunc_end" $W/t.s | awk -F: -v a=$a '$1>a{print $1; exit}')
  sed -n "${a},${b}p" $W/t.s > $W/k.s
  echo "== $v: $(grep "$K.num_vgpr" $W/t.s | awk '{print $3}') vgpr," \
       "scratch $(grep "$K.private_seg_size" $W/t.s | awk '{print $3}')"
  python3 - $W/k.s <<'EOF'
import sys
L = open(sys.argv[1]).read().split('\n')
out = []
for i, l in enumerate(L):
    s = l.strip()
    if 's_waitcnt' in s and 'vmcnt' in s: out.append(s.replace('s_waitcnt ', 'W:'))
    elif s.startswith('global_load_dwordx4'): out.append('LD')
    elif 'Loop Header: Depth=1' in s: out.append('|HDR|')
txt = ' '.join(out)
print('  ', txt[:1500])
EOF
done
