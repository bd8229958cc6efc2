#!/bin/bash
for v in $VARIANTS; do echo "== $v"; SAMPLERS_HIP_LIB=samplers_amd/lib/variants/lib_blur_$v.so timeout -k 10 100 python -u tools/blur_dbg.py || exit 1; done
