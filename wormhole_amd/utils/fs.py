"""URI resolution for every file the framework reads or writes (the dmlc
``Stream::Create`` / ``FileSystem`` surface the reference relies on,
doc/common/input.rst:53-115: local paths, ``file://``, ``hdfs://``,
``viewfs://``, ``s3://``, ``azure://``).

Local paths and ``file://`` are opened directly. A remote scheme is served
through a local mount of that filesystem (an HDFS FUSE / NFS gateway mount,
mountpoint-s3 / s3fs, blobfuse ...) named by ``WH_FS_MOUNT_<SCHEME>``:

    WH_FS_MOUNT_HDFS=/mnt/hdfs   hdfs://nn:9000/user/a/part-0 -> /mnt/hdfs/user/a/part-0
    WH_FS_MOUNT_S3=/mnt/s3       s3://bucket/key             -> /mnt/s3/bucket/key

(HDFS / viewfs drop the name-node authority, object stores keep the bucket /
container.) The native runtime resolves URIs the same way
(csrc/host/io.cc ResolvePath). A scheme without a mount is an error that
names the variable to set, never a silent local fallback.
"""
import os

_DROP_AUTHORITY = {"hdfs", "viewfs"}


def resolve(path):
    p = str(path)
    if "://" not in p:
        return p
    scheme, rest = p.split("://", 1)
    scheme_l = scheme.lower()
    if scheme_l == "file":
        return rest
    var = "WH_FS_MOUNT_" + scheme_l.upper()
    root = os.environ.get(var)
    if not root:
        raise OSError("no filesystem for '%s://' (%s): set %s to a local mount of it"
                      % (scheme, p, var))
    if scheme_l in _DROP_AUTHORITY:
        slash = rest.find("/")
        rest = rest[slash + 1:] if slash >= 0 else ""
    return os.path.join(root, rest)


def open_uri(path, mode="r", **kw):
    """open() on a resolved URI; parent directories are created for writes."""
    p = resolve(path)
    if any(c in mode for c in "wax"):
        d = os.path.dirname(p)
        if d and not os.path.isdir(d):
            os.makedirs(d, exist_ok=True)
    return open(p, mode, **kw)
