for sm in 64 128 256 512; do echo "GE_SMALL_MAX=$sm"; GE_SMALL_MAX=$sm COARSE_ONLY=40,127,500,600 timeout -k 10 300 python scripts/coarse_tune.py 2>&1 | grep us/iter; done
