#!/bin/bash
# SQ / LDS counters of pass 1 and the 3-D decoder (config 2)
scripts/pmc_kern.sh k_brick3_scan scan && scripts/pmc_kern.sh k_brick3_decode dec && scripts/pmc_kern.sh k_brick3_pack pack
