# repeat the bounded window diagnostic per library: LIBS = "prev default ic32"
cd "${GRAFT_REPO_ROOT}"
for lib in ${LIBS}; do
  for i in 1 2; do
    if [[ $lib == default ]]; then unset CPR_HIP_LIB; else export CPR_HIP_LIB=build/var/$lib.so; fi
    timeout -k 5 45 env CPR_WIN_LDS=${WIN:-0} python -u tools/dbg/win_diag2.py > gpurun_out/wr_${lib}_$i.log 2>&1
    echo "$lib $i rc=$? $(tail -1 gpurun_out/wr_${lib}_$i.log)" | tee -a gpurun_out/wr_status.log
  done
done
