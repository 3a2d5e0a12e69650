import sys

from .gpuctl import main

sys.exit(main())
