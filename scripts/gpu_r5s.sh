#!/bin/bash
export TMPDIR=/tmp
scripts/ab.sh && scripts/ab.sh --dims 280953867x1x1
