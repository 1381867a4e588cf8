#!/bin/bash
TESTS=0 SIZES=10000000 XGS="0 3 0 3 0 3" bash tools/gpu_r4w.sh
