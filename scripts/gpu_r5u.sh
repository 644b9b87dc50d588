#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 120 python scripts/c1_dec.py
