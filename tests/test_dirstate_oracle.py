"""The directory-under-removal oracle (oracle/dirstate.py), one case per reference
branch: GrainDirectoryPartition.AddSingleActivation / AddActivation / RemoveActivation /
LookUpActivations with IsValidSilo and VersionTag (GrainDirectoryPartition.cs:68-205,242-245,
274-441), LocalGrainDirectory.AdjustLocalDirectory (LocalGrainDirectory.cs:351-361) and
GrainDirectoryPartition.Merge / GrainInfo.Merge (:497-522, :139-179)."""
import dirstate as ds

M32 = ds.M32


def _k(i, tcd=3 << 56):
    return (0, i, tcd)


def test_add_single_first_wins_and_invalid_silo():
    st = ds.DirectoryState()
    st.set_valid([0, 1, 2], 4)                           # silo 3 is configured but not a member
    out = st.register([_k(1), _k(1), _k(2), _k(3)], [10, 11, 20, 30], [0, 1, 3, 9])
    assert out[0] == (10, 0, 1)                          # inserted
    assert out[1] == (10, 0, 0)                          # SingleInstance: the first registration stays (:113-117)
    assert out[2] == (M32, M32, 0)                       # IsValidSilo refuses silo 3 (:310-311)
    assert out[3] == (30, 9, 1)                          # silos past the configured range count as valid
    tag = st.entries[_k(1)][2]
    assert 0 <= tag < 1 << 31


def test_lookup_filters_invalid_silos_with_tag():
    st = ds.DirectoryState()
    st.register([_k(1), _k(2)], [10, 20], [0, 1])
    st.set_valid([0], 2)                                 # silo 1 leaves the membership
    (a1, s1, t1, f1), (a2, s2, t2, f2), (a3, _, t3, f3) = st.lookup_tagged([_k(1), _k(2), _k(7)])
    assert (a1, s1, f1) == (10, 0, 1)
    assert (a2, s2, f2) == (M32, M32, 2) and t2 == st.entries[_k(2)][2]   # empty list, the tag still returned
    assert (a3, t3, f3) == (M32, 0, 0)                   # absent: AddressesAndTag default


def test_upsert_tag_changes_only_on_change():
    st = ds.DirectoryState()
    st.upsert([_k(1)], [10], [0])
    t0 = st.entries[_k(1)][2]
    st.upsert([_k(1)], [10], [0])                        # the same activation on the same silo: no new tag
    assert st.entries[_k(1)][2] == t0
    st.upsert([_k(1), _k(1)], [11, 12], [0, 1])           # the batch's last item of a grain is applied
    assert st.entries[_k(1)][:2] == [12, 1] and st.entries[_k(1)][2] != t0
    assert st.entries[_k(1)][3] is False                  # AddActivation: not a single-instance grain


def test_unregister_needs_the_same_activation():
    st = ds.DirectoryState()
    st.register([_k(1)], [10], [0])
    assert st.unregister([_k(1)], [11]) == [0]
    assert st.unregister([_k(1)], [10]) == [1]
    assert _k(1) not in st.entries


def test_remove_silos_drops_single_keeps_multi():
    st = ds.DirectoryState()
    st.register([_k(1), _k(2), _k(3)], [10, 20, 30], [0, 1, 1])
    st.upsert([_k(4)], [ds.ACT_MULTI], [1])
    removed, multi = st.remove_silos([1])
    assert (removed, multi) == (2, 1)
    assert set(st.entries) == {_k(1), _k(4)}


def test_merge_rules():
    st = ds.DirectoryState()
    st.register([_k(1), _k(2)], [10, 20], [0, 0])
    st.upsert([_k(5)], [50], [0])                         # not single-instance
    # ActivationIds: UniqueKey.CompareTo orders by TypeCodeData, then N0, then N1
    st.set_ids([10, 11, 20, 21, 50, 51, 60], [(5, 0, 0), (4, 0, 0), (0, 1, 7), (0, 2, 7), (1, 1, 1), (1, 1, 0),
                                              (9, 9, 9)])
    keys = [_k(1), _k(2), _k(3), _k(5), _k(1 << 20)]
    acts = [11, 21, 60, 51, 20]
    silos = [2, 3, 4, 5, 6]
    tag1, tag5 = st.entries[_k(1)][2], st.entries[_k(5)][2]
    out = st.merge(keys[:4], acts[:4], silos[:4], tags=[0, 0, 123, 0])
    assert out[0] == (ds.MERGE_KEPT, 10, 0)               # incoming 11 (N0 4) < existing 10 (N0 5): the incoming stays
    assert st.entries[_k(1)][:2] == [11, 2] and st.entries[_k(1)][2] != tag1
    assert out[1] == (ds.MERGE_DROPPED, 21, 3)            # incoming 21 (N1 2) > existing 20 (N1 1): dropped
    assert st.entries[_k(2)][:2] == [20, 0]
    assert out[2] == (ds.MERGE_INSERTED, M32, M32) and st.entries[_k(3)][2] == 123   # absent: added with its tag
    # a multi-instance grain (AddActivation) holding one instance meets another: the lists are unioned
    # and both instances stay (GrainInfo.Merge :141-152, SingleInstance false): GD_ACT_MULTI, new tag
    assert out[3] == (ds.MERGE_UNION, M32, M32) and st.entries[_k(5)][0] == ds.ACT_MULTI
    assert st.entries[_k(5)][2] != tag5
    assert st.merge([_k(5)], [50], [0]) == [(ds.MERGE_HOST, M32, M32)]   # several instances now: the host's
    same = st.merge([_k(1)], [11], [2])
    assert same == [(ds.MERGE_SAME, M32, M32)]
