"""Local file cache helpers (reference hetseq/file_utils.py:1-244: ``cached_path``,
``get_from_cache``, ``url_to_filename`` for ``from_pretrained`` downloads).

This environment has no network, so remote URLs (http/https/s3) are never
fetched: ``cached_path`` resolves local paths and files already present in the
cache directory (same sha256(url)[.sha256(etag)] naming scheme as the reference,
so a cache copied from another machine is reused) and raises a clear error
otherwise.  Unlike the reference, importing this module pulls in no boto3 /
requests dependency.
"""
import hashlib
import json
import os
from urllib.parse import urlparse

PYTORCH_PRETRAINED_BERT_CACHE = os.getenv(
    'PYTORCH_PRETRAINED_BERT_CACHE', os.path.join(os.path.expanduser('~'), '.pytorch_pretrained_bert'))


def url_to_filename(url, etag=None):
    filename = hashlib.sha256(url.encode('utf-8')).hexdigest()
    if etag:
        filename += '.' + hashlib.sha256(etag.encode('utf-8')).hexdigest()
    return filename


def filename_to_url(filename, cache_dir=None):
    cache_dir = cache_dir or PYTORCH_PRETRAINED_BERT_CACHE
    meta = os.path.join(cache_dir, filename + '.json')
    if not os.path.exists(os.path.join(cache_dir, filename)) or not os.path.exists(meta):
        raise EnvironmentError('file {} not found'.format(filename))
    with open(meta, encoding='utf-8') as f:
        m = json.load(f)
    return m['url'], m.get('etag')


def get_from_cache(url, cache_dir=None):
    cache_dir = cache_dir or PYTORCH_PRETRAINED_BERT_CACHE
    if os.path.isdir(cache_dir):
        base = url_to_filename(url)
        for f in sorted(os.listdir(cache_dir)):
            if f.startswith(base) and not f.endswith('.json'):
                return os.path.join(cache_dir, f)
    raise EnvironmentError('{} is not in the local cache ({}) and this environment has no network access'
                           .format(url, cache_dir))


def cached_path(url_or_filename, cache_dir=None):
    """Local path for ``url_or_filename`` (a path, or a URL already in the cache)."""
    url_or_filename = str(url_or_filename)
    scheme = urlparse(url_or_filename).scheme
    if scheme in ('http', 'https', 's3'):
        return get_from_cache(url_or_filename, cache_dir)
    if os.path.exists(url_or_filename):
        return url_or_filename
    if scheme == '':
        raise EnvironmentError('file {} not found'.format(url_or_filename))
    raise ValueError('unable to parse {} as a URL or as a local path'.format(url_or_filename))
