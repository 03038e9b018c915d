#!/bin/bash
# round 6, final: the round-end evidence on the final code (full GPU suite,
# smoke, default bench; then the perf part: benches, kernel traces, PMC passes)
set -o pipefail
tools/round_end.sh r06zz tests && tools/round_end.sh r06zz perf
