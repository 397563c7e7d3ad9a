import json, sys
for f in sys.argv[1:]:
    t = open(f).read(); d = json.loads(t[t.index('{'):])
    print(f, d['info']['chunks'], 'kern', d['kernel_us_events'], 'span', d['span_us_stamped'], 'pro', d['prologue_us'][1],
          'loop', d['loop_us'], 'exit', d['exit_us'])
