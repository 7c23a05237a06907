#!/bin/bash
bash tools/gpu/prof_pmc.sh cfg10 --config 10
