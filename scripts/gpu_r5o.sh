#!/bin/bash
# small-slab (64-plane) brick bench A/B + full-field A/B
export TMPDIR=/tmp
scripts/ab.sh --dims 512x512x64 && scripts/ab.sh --dims 512x512x128 && scripts/ab.sh
