#!/bin/bash
# attention A/B (scripts/attn_ab.sh) then the round check (scripts/r3_check.sh); stops after a GPU fault
set -u
scripts/attn_ab.sh "$1" "$2" "${3:-attention_segments or self_attention_fullsize}"
rc=$?; [ $rc -eq 99 ] && { echo "GPU fault in the A/B: stopping"; exit 99; }
scripts/r3_check.sh "$4"
