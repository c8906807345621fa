#!/bin/bash
# r06l: round-end profiles of the final code -- rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes
# of the bench command, then the FP64 / VALU counter passes of the bench launch.
set -u
bash tools/profile_round.sh r06l || exit $?
bash tools/r05_pmc_valu.sh r06l || exit $?
