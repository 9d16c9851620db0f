# PSMNet-AA reference-order flips vs MIOpen's solver choice: the model tests, then the
# reference-order PSMNet-AA case twice more with Winograd solvers disabled (which made it
# fail every time while its plain convs ran on MIOpen).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="tests/test_gpu_models.py::test_full_model_vs_reference_golden[model_psmnet_aa-False]"
timeout -k 10 400 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread \
    tests/test_gpu_models.py -s > gpurun_out/diag_models.log 2>&1
rc=$?; echo "models rc=$rc"; grep -E "passed|failed|psmnet_aa ref-order" gpurun_out/diag_models.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  MIOPEN_DEBUG_CONV_WINOGRAD=0 timeout -k 10 200 python -m pytest -q -m gpu "$T" > gpurun_out/diag_w$i.log 2>&1
  rc=$?; echo "no-winograd run $i rc=$rc"; grep -E "AssertionError|passed|failed" gpurun_out/diag_w$i.log | head -2
  [ $rc -eq 0 ] || exit $rc
done
exit 0
