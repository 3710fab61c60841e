"""Model placement (registry.default_device): SUPER_RAG_AMD_DEVICES spreads model replicas over
GPUs request by request; SUPER_RAG_AMD_DEVICE pins one (CPU test: no encoder is built)."""


def test_devices_round_robin(monkeypatch):
    from super_rag_amd import registry
    monkeypatch.delenv("SUPER_RAG_AMD_DEVICES", raising=False)
    monkeypatch.setenv("SUPER_RAG_AMD_DEVICE", "3")
    assert [registry.default_device() for _ in range(3)] == [3, 3, 3]
    monkeypatch.setenv("SUPER_RAG_AMD_DEVICES", "0, 2,5")
    got = [registry.default_device() for _ in range(7)]
    start = [0, 2, 5].index(got[0])
    assert got == [[0, 2, 5][(start + i) % 3] for i in range(7)]
