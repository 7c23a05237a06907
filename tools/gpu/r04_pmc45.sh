#!/bin/bash
# round 4: PMC passes of configs 4 and 5 (final build)
cd $GRAFT_REPO_ROOT && bash tools/gpu/prof_pmc.sh z4 --config 4 && bash tools/gpu/prof_pmc.sh z5 --config 5 --bindings 125000
