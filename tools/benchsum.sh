#!/bin/bash
# Print value / kernel time / roofline frac of every bench JSON under gpurun_out/<tag>.
for f in gpurun_out/$1/bench*.json; do python3 -c "
import json,sys
d=json.load(open('$f')); r=d['roofline']
print('$f'.split('/')[-1], round(d['value']/1e6,2), 'M QP/s', round(r['kernel_ms']*1e3,1), 'us', 'frac', round(r['frac'],3), d['iters'])"; done
