"""Minimal S3 client for the ImageNet loader (no AWS SDK in this environment).

The reference's ImageNetLoader (src/main/scala/loaders/ImageNetLoader.scala:21-96) lists
the tar shards under a prefix with ``ListObjects`` (marker pagination), reads the labels
file and streams every shard with ``GetObject`` using profile credentials.  This module
does the same over plain HTTPS with AWS Signature Version 4:

* credentials: ``AWS_ACCESS_KEY_ID`` / ``AWS_SECRET_ACCESS_KEY`` / ``AWS_SESSION_TOKEN``,
  else the ``[AWS_PROFILE or default]`` section of ``~/.aws/credentials``
  (ProfileCredentialsProvider), else anonymous requests;
* endpoint: ``AWS_ENDPOINT_URL`` / ``endpoint=`` (path-style addressing, e.g. a MinIO or
  on-prem gateway), else ``https://<bucket>.s3.<region>.amazonaws.com``.
"""
from __future__ import annotations

import configparser
import datetime as _dt
import hashlib
import hmac
import os
import urllib.parse
import urllib.request
import xml.etree.ElementTree as ET

EMPTY_SHA = hashlib.sha256(b"").hexdigest()


def parse_url(url: str) -> tuple[str, str]:
    """``s3://bucket/key`` -> (bucket, key)."""
    u = urllib.parse.urlparse(url)
    if u.scheme != "s3":
        raise ValueError(f"not an s3:// URL: {url!r}")
    return u.netloc, u.path.lstrip("/")


def _credentials():
    ak, sk = os.environ.get("AWS_ACCESS_KEY_ID"), os.environ.get("AWS_SECRET_ACCESS_KEY")
    if ak and sk:
        return ak, sk, os.environ.get("AWS_SESSION_TOKEN")
    path = os.environ.get("AWS_SHARED_CREDENTIALS_FILE", os.path.expanduser("~/.aws/credentials"))
    if os.path.exists(path):
        cp = configparser.ConfigParser()
        cp.read(path)
        prof = os.environ.get("AWS_PROFILE", "default")
        if cp.has_section(prof):
            sec = cp[prof]
            if "aws_access_key_id" in sec and "aws_secret_access_key" in sec:
                return sec["aws_access_key_id"], sec["aws_secret_access_key"], sec.get("aws_session_token")
    return None


def _sign(key: bytes, msg: str) -> bytes:
    return hmac.new(key, msg.encode(), hashlib.sha256).digest()


def sigv4_headers(method: str, url: str, region: str, creds, now: _dt.datetime | None = None,
                  payload_sha: str = EMPTY_SHA, extra: dict | None = None) -> dict:
    """Headers of an AWS SigV4-signed request (service ``s3``); ``extra`` headers are
    sent and signed too."""
    u = urllib.parse.urlparse(url)
    now = now or _dt.datetime.now(_dt.timezone.utc)
    amz_date = now.strftime("%Y%m%dT%H%M%SZ")
    date = amz_date[:8]
    headers = {"host": u.netloc, "x-amz-content-sha256": payload_sha, "x-amz-date": amz_date}
    headers.update({k.lower(): v for k, v in (extra or {}).items()})
    if creds is None:
        return headers
    ak, sk, token = creds
    if token:
        headers["x-amz-security-token"] = token
    q = urllib.parse.parse_qsl(u.query, keep_blank_values=True)
    canon_q = "&".join(f"{urllib.parse.quote(k, safe='-_.~')}={urllib.parse.quote(v, safe='-_.~')}"
                       for k, v in sorted(q))
    names = sorted(headers)
    canon_h = "".join(f"{n}:{headers[n].strip()}\n" for n in names)
    signed = ";".join(names)
    path = urllib.parse.quote(u.path or "/", safe="/-_.~%")
    creq = "\n".join([method, path, canon_q, canon_h, signed, payload_sha])
    scope = f"{date}/{region}/s3/aws4_request"
    sts = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope, hashlib.sha256(creq.encode()).hexdigest()])
    k = _sign(_sign(_sign(_sign(("AWS4" + sk).encode(), date), region), "s3"), "aws4_request")
    sig = hmac.new(k, sts.encode(), hashlib.sha256).hexdigest()
    headers["Authorization"] = f"AWS4-HMAC-SHA256 Credential={ak}/{scope}, SignedHeaders={signed}, Signature={sig}"
    return headers


class S3Client:
    def __init__(self, region: str | None = None, endpoint: str | None = None, timeout: float = 60.0):
        self.region = region or os.environ.get("AWS_REGION", os.environ.get("AWS_DEFAULT_REGION", "us-east-1"))
        self.endpoint = (endpoint or os.environ.get("AWS_ENDPOINT_URL") or "").rstrip("/")
        self.creds = _credentials()
        self.timeout = timeout

    def _url(self, bucket: str, key: str = "", query: dict | None = None) -> str:
        qk = urllib.parse.quote(key, safe="/-_.~")
        base = (f"{self.endpoint}/{bucket}/{qk}" if self.endpoint
                else f"https://{bucket}.s3.{self.region}.amazonaws.com/{qk}")
        if query:
            base += "?" + urllib.parse.urlencode(sorted(query.items()), quote_via=urllib.parse.quote)
        return base

    def _open(self, url: str):
        req = urllib.request.Request(url, headers=sigv4_headers("GET", url, self.region, self.creds))
        return urllib.request.urlopen(req, timeout=self.timeout)

    def list_objects(self, bucket: str, prefix: str = "") -> list[str]:
        """All keys under ``prefix`` (ListObjects with marker pagination)."""
        keys, marker = [], ""
        while True:
            q = {"prefix": prefix}
            if marker:
                q["marker"] = marker
            with self._open(self._url(bucket, "", q)) as r:
                root = ET.fromstring(r.read())
            ns = root.tag[:root.tag.index("}") + 1] if root.tag.startswith("{") else ""
            page = [c.findtext(f"{ns}Key") for c in root.findall(f"{ns}Contents")]
            keys += page
            if (root.findtext(f"{ns}IsTruncated") or "false").lower() != "true":
                return keys
            marker = root.findtext(f"{ns}NextMarker") or (page[-1] if page else "")
            if not marker:
                return keys

    def get_object(self, bucket: str, key: str):
        """A readable binary stream of the object."""
        return self._open(self._url(bucket, key))
