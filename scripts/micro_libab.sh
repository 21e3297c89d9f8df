# Alternating micro-benchmark of two library builds on the one-pass kernel:
#   bash scripts/micro_libab.sh OLD.so NEW.so N ANGLES REPS VARIANTS  (F32=1 for fp32)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r4}; mkdir -p $O; : > $O/micro_libab.jsonl
for r in 1 2; do
  for lib in "$1" "$2"; do
    HGM_LIB=$lib HGM_MICRO_F32=${F32:-0} timeout -k 10 300 python -u scripts/fused_micro.py $3 $4 $5 $6 2>/dev/null | grep variant | sed "s|^{|{\"lib\": \"$lib\", |" | tee -a $O/micro_libab.jsonl || exit 1
  done
done
