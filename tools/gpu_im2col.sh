set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/im2col; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -k "im2col or e2e or embed" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -2 $O/pytest.log
bash tools/lib_ab.sh ab/libaaclip_base.so aa-clip_amd/aaclip/libaaclip_hip.so 2>&1 | tee $O/lib_ab.txt || exit 4
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 5; }
python -c "import json; d=json.load(open('$O/bench.json')); p=d['step_profile']; print(d['value'], p['one_stream']['by_op']['im2col'], p['timed_streams']['by_op']['im2col'])"
