"""Batch driver: BatchRun.m without the folder-picker GUI.

``find_folders`` restates BatchRun.m's ``findfiles`` (BatchRun.m:71-150): a folder qualifies when it
holds one each of .pho/.ext/.cnt/.int; a folder holding some but not all of them is reported and
skipped; a second file of an extension already seen prints a warning and clears the list of found
extensions (the reference's ``found = []``, BatchRun.m:92-96); subfolders are searched recursively
after the folder's own files.  ``batch_run`` calls ``main(folder)`` for each qualifying folder in order
and stops at the first failure (BatchRun.m:56-64).
"""
import os
import sys

EXTS = (".pho", ".ext", ".cnt", ".int")


def _join(items):
    return ", ".join(items[:-1]) + " and " + items[-1] if len(items) > 1 else items[0]


def find_folders(folder, exts=EXTS, log=print):
    """BatchRun.m:71-150 (files in name order, as MATLAB's dir lists them)."""
    out = []
    try:
        entries = sorted(os.listdir(folder))
    except OSError:
        return out
    files = [e for e in entries if os.path.isfile(os.path.join(folder, e))]
    if files:
        found = []
        for name in files:
            ext = os.path.splitext(name)[1]
            if ext in exts:
                if ext in found:
                    log(f"Warning: More than 1 {ext} file was found in {folder}")
                    found = []
                found.append(ext)
        if found and len(found) < len(exts):
            missing = [e for e in sorted(exts) if e not in found]  # setdiff returns sorted values
            log(f'Error: {_join(found)} {"were" if len(found) > 1 else "was"} found in "{folder}" but not '
                f"{_join(missing)}. This folder will be skipped")
        elif len(found) == len(exts):
            out.append(folder)
    for name in entries:
        sub = os.path.join(folder, name)
        if os.path.isdir(sub):
            out.extend(find_folders(sub, exts, log))
    return out


def batch_run(paths, device=0):
    """BatchRun.m:42-66: every data folder under the selected paths through main(folder, false);
    stops at the first folder whose main() fails.  Returns the list of (folder, main_error)."""
    from .bundle import main
    folders = []
    for p in paths:
        folders.extend(find_folders(p))
    done = []
    for f in folders:
        err = main(f, False, device=device)
        done.append((f, err))
        if err == 1:
            break
    return done


def cli(argv=None):
    """python -m fba_cli main <folder> | batch <folder>...   (main(folder, plot) / BatchRun.m)"""
    argv = list(sys.argv[1:] if argv is None else argv)
    if len(argv) >= 2 and argv[0] == "main":
        from .bundle import main
        return main(argv[1], len(argv) > 2 and argv[2] not in ("0", "false"))
    if len(argv) >= 2 and argv[0] == "batch":
        done = batch_run(argv[1:])
        return 1 if any(e for _, e in done) else 0
    print("usage: fba_cli.py main <folder> [plot] | batch <folder>...")
    return 2
