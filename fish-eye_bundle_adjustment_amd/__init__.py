"""MI355X-native Gauss-Newton bundle-adjustment inner loop.

A drop-in for the hot path of wynandtredoux/Fish-Eye_Bundle_Adjustment (MATLAB): BuildAwG ->
A'PA / A'Pw -> bordered solve -> xhat update, implemented as hand-written HIP kernels for gfx950
behind the C-ABI in ``include/fba.h`` (``libfba.so``).  This package is the host-side mirror of the
reference's interface (file formats, ``main(folder, plot)``, ``Buildxhat`` / ``BuildAwG`` /
``BuildRSD``).  The directory name contains hyphens, so it is loaded under the module name
``fba_amd`` (see ``fba_import.py`` at the repository root).
"""
from . import capi
from .capi import Context, FBAError
from .io import Dataset, IngestError, load_folder, xhat_names
from .bundle import Adjustment, BuildAwG, Buildxhat, BuildRSD, adjust, main, write_outputs

__all__ = ["capi", "Context", "FBAError", "Dataset", "IngestError", "load_folder", "xhat_names", "Adjustment",
           "BuildAwG", "Buildxhat", "BuildRSD", "adjust", "main", "write_outputs"]
