import sys

from cain_amd.runner.cli import main

if __name__ == "__main__":
    sys.exit(main())
