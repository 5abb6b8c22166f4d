#!/usr/bin/env python3
"""Command line for the reference's two entry points on the MI355X path:

    python fba_cli.py main <folder> [plot]     main(folder, plot)  (main.m:10)
    python fba_cli.py batch <folder>...        BatchRun.m without its folder picker
"""
import sys

import fba_import

if __name__ == "__main__":
    fba = fba_import.load()
    from fba_amd.batch import cli
    sys.exit(cli())
