for g in 16 32 64; do echo "G=$g"; GE_GRP_G=$g COARSE_ONLY=2000,5000 timeout -k 10 300 python scripts/coarse_tune.py 2>&1 | grep us/iter; done
