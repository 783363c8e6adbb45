"""Download cache for pretrained archives and vocabularies (reference hetseq/file_utils.py:1-244:
``cached_path``, ``get_from_cache``, ``http_get``, ``s3_get``, ``s3_etag``, ``url_to_filename``,
``filename_to_url``, ``split_s3_path``, ``read_set_from_file``, ``get_file_extension``).

Same cache layout as the reference -- ``sha256(url)[.sha256(etag)]`` plus a ``.json`` with
``{"url", "etag"}`` -- so a cache populated by the reference (or copied from another machine) is
reused as is.  Differences, all for multi-process training jobs:

* HTTP(S) through the standard library (``urllib``): no ``requests`` / ``boto3`` import at module
  load; S3 needs ``boto3`` only when an ``s3://`` URL is actually fetched.
* The download goes to a temporary file IN the cache directory and is renamed into place
  (``os.replace``): a reader never sees a partial file, and the ``.json`` is written before the
  rename, so an entry that exists is complete.
* One downloader per entry: the ranks of a job that resolve the same URL at once serialise on an
  ``fcntl`` lock file next to the entry; the others find the finished file.
* No network (or the server down): ``get_from_cache`` falls back to the newest cached copy of the
  URL (any ETag) instead of failing -- the reference raises on the HEAD request.
"""
import fcntl
import hashlib
import json
import logging
import os
import shutil
import tempfile
import urllib.error
import urllib.request
from functools import wraps
from urllib.parse import urlparse

logger = logging.getLogger(__name__)

PYTORCH_PRETRAINED_BERT_CACHE = os.getenv(
    'PYTORCH_PRETRAINED_BERT_CACHE', os.path.join(os.path.expanduser('~'), '.pytorch_pretrained_bert'))

_TIMEOUT = float(os.getenv('HX_DOWNLOAD_TIMEOUT', '60'))


def url_to_filename(url, etag=None):
    """``sha256(url)``, plus ``.sha256(etag)`` when the server gave an ETag (reference layout)."""
    filename = hashlib.sha256(url.encode('utf-8')).hexdigest()
    if etag:
        filename += '.' + hashlib.sha256(etag.encode('utf-8')).hexdigest()
    return filename


def filename_to_url(filename, cache_dir=None):
    """The (url, etag) stored for cache entry ``filename``; EnvironmentError if either file is missing."""
    cache_dir = str(cache_dir or PYTORCH_PRETRAINED_BERT_CACHE)
    path = os.path.join(cache_dir, filename)
    if not os.path.exists(path):
        raise EnvironmentError('file {} not found'.format(path))
    meta = path + '.json'
    if not os.path.exists(meta):
        raise EnvironmentError('file {} not found'.format(meta))
    with open(meta, encoding='utf-8') as f:
        m = json.load(f)
    return m['url'], m.get('etag')


def split_s3_path(url):
    """``s3://bucket/key`` -> (bucket, key)."""
    parsed = urlparse(url)
    if not parsed.netloc or not parsed.path:
        raise ValueError('bad s3 path {}'.format(url))
    return parsed.netloc, parsed.path.lstrip('/')


def _boto3():
    try:
        import boto3  # noqa: F401
        from botocore.exceptions import ClientError  # noqa: F401
    except ImportError as e:
        raise EnvironmentError('s3:// URLs need boto3, which is not installed') from e
    return boto3, ClientError


def s3_request(func):
    """Turn a botocore 404 into EnvironmentError('file ... not found') (reference wrapper)."""
    @wraps(func)
    def wrapper(url, *args, **kwargs):
        _, client_error = _boto3()
        try:
            return func(url, *args, **kwargs)
        except client_error as exc:
            if str(exc.response.get('Error', {}).get('Code')) in ('404', 'NoSuchKey'):
                raise EnvironmentError('file {} not found'.format(url)) from exc
            raise
    return wrapper


@s3_request
def s3_etag(url):
    boto3, _ = _boto3()
    bucket, key = split_s3_path(url)
    return boto3.resource('s3').Object(bucket, key).e_tag


@s3_request
def s3_get(url, temp_file):
    boto3, _ = _boto3()
    bucket, key = split_s3_path(url)
    boto3.resource('s3').Bucket(bucket).download_fileobj(key, temp_file)


def http_etag(url, timeout=None):
    """ETag from a HEAD request (redirects followed); IOError on a non-200 answer."""
    req = urllib.request.Request(url, method='HEAD')
    try:
        with urllib.request.urlopen(req, timeout=timeout or _TIMEOUT) as r:
            return r.headers.get('ETag')
    except urllib.error.HTTPError as e:
        raise IOError('HEAD request failed for url {} with status code {}'.format(url, e.code)) from e


def http_get(url, temp_file, timeout=None, progress=None):
    """Stream ``url`` into the open binary file ``temp_file`` (1 MB chunks; a tqdm bar when
    ``progress`` is true and tqdm is importable)."""
    with urllib.request.urlopen(url, timeout=timeout or _TIMEOUT) as r:
        total = r.headers.get('Content-Length')
        bar = None
        if progress:
            try:
                from tqdm import tqdm
                bar = tqdm(unit='B', unit_scale=True, total=int(total) if total is not None else None)
            except ImportError:
                bar = None
        n = 0
        while True:
            chunk = r.read(1 << 20)
            if not chunk:
                break
            temp_file.write(chunk)
            n += len(chunk)
            if bar is not None:
                bar.update(len(chunk))
        if bar is not None:
            bar.close()
    if total is not None and n != int(total):
        raise IOError('download of {} truncated: {} of {} bytes'.format(url, n, total))
    return n


def _cached_copies(cache_dir, url):
    """Existing complete entries of ``url`` (any ETag), newest first."""
    if not os.path.isdir(cache_dir):
        return []
    base = url_to_filename(url)
    out = [os.path.join(cache_dir, f) for f in os.listdir(cache_dir)
           if (f == base or f.startswith(base + '.')) and not f.endswith(('.json', '.lock', '.part'))]
    return sorted(out, key=os.path.getmtime, reverse=True)


def get_from_cache(url, cache_dir=None, progress=False):
    """Path of the cached copy of ``url``, downloading it first if this ETag is not cached yet."""
    cache_dir = str(cache_dir or PYTORCH_PRETRAINED_BERT_CACHE)
    os.makedirs(cache_dir, exist_ok=True)
    try:
        etag = s3_etag(url) if url.startswith('s3://') else http_etag(url)
    except (urllib.error.URLError, OSError) as e:
        # HTTP errors that are answers (404, 403, ...) are the caller's problem, not connectivity
        if isinstance(e, IOError) and 'status code' in str(e):
            raise
        copies = _cached_copies(cache_dir, url)
        if copies:
            logger.warning('%s unreachable (%s): using the cached copy %s', url, e, copies[0])
            return copies[0]
        raise EnvironmentError('{} is not reachable ({}) and not in the cache {}'.format(url, e, cache_dir)) from e
    path = os.path.join(cache_dir, url_to_filename(url, etag))
    if os.path.exists(path):
        return path
    with open(path + '.lock', 'w') as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)   # one downloader; the others wait and find the file
        try:
            if os.path.exists(path):
                return path
            logger.info('%s not found in cache, downloading to %s', url, path)
            fd, tmp = tempfile.mkstemp(dir=cache_dir, suffix='.part')
            try:
                with os.fdopen(fd, 'wb') as f:
                    if url.startswith('s3://'):
                        s3_get(url, f)
                    else:
                        http_get(url, f, progress=progress)
                with open(path + '.json', 'w', encoding='utf-8') as m:
                    json.dump({'url': url, 'etag': etag}, m)
                os.replace(tmp, path)
            finally:
                if os.path.exists(tmp):
                    os.remove(tmp)
        finally:
            fcntl.flock(lock, fcntl.LOCK_UN)
    return path


def cached_path(url_or_filename, cache_dir=None):
    """A URL (http, https, s3) -> the path of its cached download; a path -> itself if it exists."""
    url_or_filename = str(url_or_filename)
    scheme = urlparse(url_or_filename).scheme
    if scheme in ('http', 'https', 's3'):
        return get_from_cache(url_or_filename, cache_dir)
    if os.path.exists(url_or_filename):
        return url_or_filename
    if scheme == '':
        raise EnvironmentError('file {} not found'.format(url_or_filename))
    raise ValueError('unable to parse {} as a URL or as a local path'.format(url_or_filename))


def read_set_from_file(filename):
    """The set of lines (right-stripped) of a text file."""
    with open(filename, 'r', encoding='utf-8') as f:
        return {line.rstrip() for line in f}


def get_file_extension(path, dot=True, lower=True):
    ext = os.path.splitext(path)[1]
    ext = ext if dot else ext[1:]
    return ext.lower() if lower else ext


def copy_to_cache(src, url, etag=None, cache_dir=None):
    """Install a local file as the cache entry of ``url`` (seeding an offline machine's cache)."""
    cache_dir = str(cache_dir or PYTORCH_PRETRAINED_BERT_CACHE)
    os.makedirs(cache_dir, exist_ok=True)
    path = os.path.join(cache_dir, url_to_filename(url, etag))
    with open(path + '.json', 'w', encoding='utf-8') as m:
        json.dump({'url': url, 'etag': etag}, m)
    shutil.copyfile(src, path)
    return path
