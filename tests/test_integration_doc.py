"""CPU: INTEGRATION.md quotes the reference-side bodies that tests/test_gpu_refside.py runs
(examples/refside/solver_bodies.cpp) verbatim, and every body is quoted."""
import os
import sys

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_integration_doc_quotes_the_compiled_bodies():
    import integration_bodies as IB
    src, doc = IB.bodies(), IB.doc_blocks()
    assert set(src) == {"Random", "Extractor", "Frame", "Matcher::match", "RansacSE3", "Gicp", "PnPRansac::compute",
                        "Frame::createFilteredCloud", "Tracking::createKeyFrame"}
    assert set(doc) == set(src), (sorted(doc), sorted(src))
    for k in src:
        assert doc[k] == src[k], f"INTEGRATION.md block {k!r} differs from solver_bodies.cpp (tools/integration_bodies.py)"


def test_reference_members_used_by_the_bodies():
    """The bodies use the reference's member names (Solver/Solver.h:22-25, Solver/Gicp.h:34-46) and none of
    the names the round-4 doc invented."""
    import integration_bodies as IB
    text = "".join(IB.bodies().values())
    for name in ("mF1", "mF2", "mMatches", "mbUpdate", "mGuess", "mT", "setOutlier", "setInlier", "mvInliers", "mT21"):
        assert name in text, name
    # the Frame members the reference's callers read (Core/Frame.cpp:34-117; Tracking.cpp:101-111,158; PoseGraph)
    frame = IB.bodies()["Frame"]
    for name in ("mnId = nNextId++", "mImColor(imRGB)", "cvtColor(imRGB, mImGray", "convertTo(mImDepth, CV_32F",
                 "mvpLandmarks", "mvbOutlier", "computeImageBounds()", "assignFeaturesToGrid()", "mvKeysColor"):
        assert name in frame, name
    # the solvers take the calling thread's context (the PoseGraph thread runs Matcher / RansacSE3 too)
    assert "std::this_thread::get_id()" in IB.bodies()["Extractor"]
    assert "Random::mutex()" in IB.bodies()["RansacSE3"]
    for bad in ("mvMatches", "mpF1", "mpF2", "mMaxIterations", "mMaxCorrDist"):
        assert bad not in text, bad
