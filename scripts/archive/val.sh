#!/bin/bash
# usage: scripts/val.sh TAG [ENV=V ...] -- bench args : print "TAG value ms_per_step" of one bench.py run
tag=$1; shift
envs=()
while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
env "${envs[@]}" timeout -k 10 300 python bench.py "$@" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'])"
