# Per-kernel VALU instruction histograms of tools/isa_fe_variants.hip (compile only, no GPU).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${TMPDIR:-/tmp}/isa_fe_variants.s
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I"$ROOT/eges_amd/csrc" --offload-device-only -S \
  -o "$OUT" "$ROOT/tools/isa_fe_variants.hip" 2>/dev/null
for k in k_mul_schoolbook k_mul_karatsuba k_sqr; do
  echo "== $k"
  awk "/^_Z[0-9]*${k}/,/s_endpgm/" "$OUT" | grep -E "^\s+v_" | awk '{print $1}' | sort | uniq -c | sort -rn | head -12
done
