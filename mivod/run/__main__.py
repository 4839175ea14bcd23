import sys

from .launcher import main

sys.exit(main())
