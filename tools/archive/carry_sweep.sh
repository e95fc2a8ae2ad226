cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/carry
mkdir -p $O
timeout -k 10 300 python tools/seeds.py $O/euro252_c2.jsonl 1-16 --steps 2 --warmup 1 --preset euro252 --lm-lam-carry 2 > $O/a.log 2>&1 || exit 1
timeout -k 10 300 python tools/seeds.py $O/euro30_c2.jsonl 1-16 --steps 2 --warmup 1 --preset euro30 --lm-lam-carry 2 > $O/b.log 2>&1 || exit 1
timeout -k 10 300 python tools/seeds.py $O/heston30_c2.jsonl 1-16 --steps 2 --warmup 1 --preset heston30 --lm-lam-carry 2 > $O/c.log 2>&1 || exit 1
python tools/seed_summary.py $O/*.jsonl
