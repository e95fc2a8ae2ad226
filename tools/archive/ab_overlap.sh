for a in "RPH_LM_GRAM_OVERLAP=0|" "RPH_LM_GRAM_OVERLAP=1|" "RPH_LM_GRAM_OVERLAP=0|--lm-leaf-paths 1024" "RPH_LM_GRAM_OVERLAP=1|--lm-leaf-paths 1024" "RPH_LM_GRAM_OVERLAP=0|" "RPH_LM_GRAM_OVERLAP=1|"; do
  e=${a%%|*}; f=${a#*|}
  env $e timeout -k 10 100 python bench.py --steps 20 --warmup 3 $f > /tmp/o.json || exit 1
  python -c "import json; d=json.loads(open('/tmp/o.json').read()); print('$e $f', round(d['ms_per_step'],4), d['quality']['terminal_pnl_std'])"
done
