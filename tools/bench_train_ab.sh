#!/bin/bash
# Training bench A/B in one box session: the working tree vs a copy of it whose pnr/train.py
# (or AB_FILE=pnr/<name>.py) is replaced by pixel-nerf_amd/build/old_<name>.py (written
# locally from a git revision).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OLD=/tmp/pnr_old_repo
F=${AB_FILE:-pnr/train.py}
rm -rf $OLD && cp -r . $OLD && cp pixel-nerf_amd/build/old_$(basename $F) $OLD/pixel-nerf_amd/$F || exit 1
for round in 1 2; do
  for v in old new; do
    root=.; [ $v = old ] && root=$OLD
    echo -n "$v: "
    timeout -k 10 300 python $root/scripts/bench_train.py --steps 10 --warmup 3 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" || exit $?
  done
done
