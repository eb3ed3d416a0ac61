"""UiConnectionInfo, after the reference's UiConnectionInfoTest (deeplearning4j-core/src/test/java/org/deeplearning4j/
ui/UiConnectionInfoTest.java:14-110): scheme / address / port prefix and normalised path parts. CPU."""
import pytest

from deeplearning4j_amd.ui import UiConnectionInfo


def _b():
    return UiConnectionInfo.Builder().setAddress("192.168.1.1").enableHttps(True).setPort(8082)


def test_first_part():
    assert UiConnectionInfo.Builder().setPort(8080).build().getFirstPart() == "http://localhost:8080"
    assert UiConnectionInfo.Builder().enableHttps(True).setPort(8080).build().getFirstPart() == "https://localhost:8080"
    assert _b().build().getFirstPart() == "https://192.168.1.1:8082"


@pytest.mark.parametrize("path,sub,expect", [("www-data", None, "/www-data/"), ("/www-data/tmp/", None, "/www-data/tmp/"),
                                             ("/www-data/tmp", None, "/www-data/tmp/"),
                                             ("/www-data//tmp", None, "/www-data/tmp/"),
                                             ("/www-data//tmp", "alpha", "/www-data/tmp/alpha/"),
                                             ("//www-data//tmp", "/alpha/", "/www-data/tmp/alpha/"),
                                             ("//www-data//tmp", "/alpha//beta/", "/www-data/tmp/alpha/beta/")])
def test_second_part(path, sub, expect):
    info = _b().setPath(path).build()
    assert (info.getSecondPart(sub) if sub else info.getSecondPart()) == expect


def test_full_address():
    info = UiConnectionInfo.Builder().setAddress("192.168.1.1").enableHttps(False).setPort(8082) \
        .setPath("/www-data//tmp").build()
    assert info.getFullAddress() == "http://192.168.1.1:8082/www-data/tmp/"
