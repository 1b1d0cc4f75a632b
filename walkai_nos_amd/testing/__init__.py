"""Test helpers for nos users and for this repository's own suites (reference ``pkg/test``):
fluent object builders (``factory``) and recording fakes of the device-side clients (``mocks``)."""
from .factory import NodeBuilder, PodBuilder, build_namespace  # noqa: F401
from .mocks import MockDevicePluginClient, MockNodeInitializer, MockPartitionClient, RecordingBarrier  # noqa: F401
