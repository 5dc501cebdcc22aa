#!/bin/bash
# Round 5: the full GPU suite and smoke() on the final code.
source scripts/gpu_step.sh
step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
