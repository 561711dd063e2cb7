import sys

from kubedl_amd.cli.main import main

sys.exit(main())
