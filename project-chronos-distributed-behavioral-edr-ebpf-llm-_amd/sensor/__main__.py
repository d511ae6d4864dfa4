import sys

from .main import run

sys.exit(run())
