"""Build metadata: application version and build number.

The reference stamps ``buildmeta.AppVersion`` and ``buildmeta.BuildNumber`` into the
binary at link time (``-ldflags -X …``, ``/root/reference/.container/Dockerfile:14``),
from the ``APPVERSION`` / ``BUILDNUMBER`` build args its image workflow computes
(``/root/reference/.github/workflows/build-image.yaml:31-70``).  A Python package has
no link step, so the image build writes them into ``_buildinfo.py`` next to this
module instead (``python -m nexus_supervisor_amd.buildmeta --write VERSION BUILD``,
``deploy/Dockerfile*``); a source checkout reports ``DEFAULT_VERSION`` / ``dev``.
The version is what ``python -m nexus_supervisor_amd version`` prints, what the
``version`` metric tag carries and what the start-up log line reports.
"""
from __future__ import annotations

import os
import re
import sys

DEFAULT_VERSION = "0.1.0"

try:  # written at image build
    from ._buildinfo import APP_VERSION, BUILD_NUMBER  # type: ignore[import-not-found]
except ImportError:
    APP_VERSION, BUILD_NUMBER = DEFAULT_VERSION, "dev"

_SEMVER = re.compile(r"^v?(\d+)\.(\d+)\.(\d+)(?:[-+][0-9A-Za-z.+-]+)?$")


def write(version: str, build: str, path: str = "") -> str:
    """Stamp the build (image build step).  ``version`` must be semver (``v`` prefix ok)."""
    if not _SEMVER.match(version):
        raise ValueError(f"not a semantic version: {version!r}")
    if not re.fullmatch(r"[0-9A-Za-z._-]+", build):
        raise ValueError(f"bad build number: {build!r}")
    path = path or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_buildinfo.py")
    with open(path, "w") as f:
        f.write(f'"""Generated at image build by nexus_supervisor_amd.buildmeta."""\n'
                f"APP_VERSION = {version.lstrip('v')!r}\nBUILD_NUMBER = {build!r}\n")
    return path


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if len(argv) == 3 and argv[0] == "--write":
        print(write(argv[1], argv[2]))
        return 0
    print(f"{APP_VERSION} (build {BUILD_NUMBER})")
    return 0


if __name__ == "__main__":
    sys.exit(main())
