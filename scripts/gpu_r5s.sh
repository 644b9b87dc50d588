#!/bin/bash
export TMPDIR=/tmp
scripts/ab.sh
