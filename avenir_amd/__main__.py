import sys

from . import freeze_startup_objects
from .cli import main

freeze_startup_objects()
sys.exit(main())
