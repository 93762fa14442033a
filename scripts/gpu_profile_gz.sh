# scripts/gpu_profile_all.sh, then its CSVs gzipped (a c5 / cadence PMC pass holds a row per
# dispatch: tens of MB, past what gpurun copies back); gunzip them before summarize_round.py
cd $GRAFT_REPO_ROOT && bash scripts/gpu_profile_all.sh "$@" && find gpurun_out/prof_$1 -name "*.csv" -exec gzip -9 {} + && echo "gz=0"
