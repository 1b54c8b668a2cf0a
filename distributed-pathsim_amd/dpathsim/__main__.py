"""``python -m dpathsim`` -- see dpathsim.cli."""
import sys

from .cli import main

sys.exit(main())
