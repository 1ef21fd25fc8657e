#!/bin/bash
# final-tree check: full GPU suite and the driver's smoke()
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/s12_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s12_smoke.log 2>&1 || exit 1
echo S12_DONE
