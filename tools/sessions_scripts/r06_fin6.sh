#!/usr/bin/env bash
# round 6: the committed tree's whole GPU suite and smoke, once more (tests added after fin5)
tools/gpu_session.sh r06_fin6 \
  "700|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "100|python3 -c 'import __graft_entry__ as g; g.smoke()'"
