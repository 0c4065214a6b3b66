#!/bin/bash
# A/B: config 2's small sizes with the copy launches enqueued one by one vs
# replayed from one hipGraph (MPX_COPY_GRAPH=1), two interleaved passes.
# The graph lost (profiles/r01_copy_graph_ab.jsonl) and the temporary
# MPX_COPY_GRAPH knob in mpx_copy was removed; the script records the method.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/copy_graph.jsonl
: > $out
for pass in 1 2; do
    for g in 0 1; do
        for n in 16 4096 65536 1048576 4194304 16777216 1073741824; do
            MPX_COPY_GRAPH=$g timeout -k 10 60 python -u tools/copy_sweep.py one $n | sed "s/^{/{\"graph\": $g, /" >> $out || exit $?
        done
    done
done
echo done
