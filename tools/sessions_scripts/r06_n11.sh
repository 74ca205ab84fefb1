#!/usr/bin/env bash
# round 6: measured HBM traffic per round of a narrow cfg4 run (FETCH_SIZE / WRITE_SIZE per dispatch,
# tools/pmc_cfg5.sh's passes over tools/bench_configs.py cfg4 with ACSIM_BIN_NARROW=1): the 8-byte
# rounds against the 4-byte ones
tools/gpu_session.sh r06_n11 \
  "300|ACSIM_BIN_NARROW=1 CFG=cfg4 tools/pmc_cfg5.sh r06_n11/pmc"
