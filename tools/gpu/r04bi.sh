# round 4 final checkpoint: full GPU suite, smoke, default bench (rec128 headline)
mkdir -p gpurun_out/r04bi
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r04bi/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as G; G.smoke(); print('smoke ok')" > gpurun_out/r04bi/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r04bi/bench.json 2> gpurun_out/r04bi/bench.err || exit 1
