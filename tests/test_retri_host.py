"""Host-side contract of processors/track_retriangulation.py that needs no GPU."""
import pytest

from instantsfm_amd.processors import track_retriangulation as TR


def test_merge_tracks_raises_like_the_reference():
    """The reference's merge_tracks (track_retriangulation.py:110-198) cannot run: it uses faiss.IndexFlatL2 (:136)
    without importing faiss (:1-14), and its only call is commented out (:210-212).  Ours raises with that reason
    instead of a NameError, before touching the scene."""
    tracks = {0: object()}
    with pytest.raises(NotImplementedError, match="faiss"):
        TR.merge_tracks([], [], tracks, {"merge_max_reproj_error": 4.0})
    assert list(tracks) == [0]
