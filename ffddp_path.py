"""Puts the product package directory (franka-force-feedback-mpc_amd/, whose
name is not a Python identifier) on sys.path so `import ffddp` works."""
import sys
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent / "franka-force-feedback-mpc_amd"
if str(PKG_DIR) not in sys.path:
    sys.path.insert(0, str(PKG_DIR))
