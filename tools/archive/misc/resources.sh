#!/bin/bash
# Print VGPR / SGPR / scratch / occupancy per kernel from the asm build.
make -s -C "$(dirname "$0")/../reticulum_amd/csrc" asm 2>&1 | grep -E "error|Function Name|VGPRs:|TotalSGPRs|ScratchSize|Occupancy" \
 | sed -E 's/.*remark: +//; s/ \[-Rpass-analysis=kernel-resource-usage\]//' | sed -E "s/reticulum_amd[^ ]*: +//g" | paste - - - - - \
 | sed -E 's/Function Name: _ZN6rnstok//; s/EEEvNS_[0-9]+[A-Za-z]+E//'
