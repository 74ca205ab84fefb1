#!/usr/bin/env bash
# round 6: randomized narrow-plan parity (tests/test_properties.py::test_gpu_narrow_random_configs)
tools/gpu_session.sh r06_n10 \
  "500|python -u -m pytest tests/test_properties.py -k narrow -x -v --hypothesis-show-statistics --timeout 400 --timeout-method thread"
