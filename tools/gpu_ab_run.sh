#!/bin/bash
# A/B of tile-schedule variants of the cfg2 bench (dev tool): kernel traces per variant.
export VARIANTS="${VARIANTS:-def MPCQ_X=0
occ8 MPCQ_TILE_OCC=8}"
export TRACE=1
bash tools/ab_env.sh
