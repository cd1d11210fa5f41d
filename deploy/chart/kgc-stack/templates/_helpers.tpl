{{- define "kgc.engineImage" -}}
{{- $repo := .ms.repository | default .root.Values.engineImage.repository -}}
{{- if or (hasPrefix "vllm/" $repo) (contains "vllm-openai" $repo) -}}
{{ .root.Values.engineImage.repository }}:{{ .root.Values.engineImage.tag }}
{{- else -}}
{{ $repo }}:{{ .ms.tag | default .root.Values.engineImage.tag }}
{{- end -}}
{{- end -}}

{{- define "kgc.gpus" -}}
{{- $vc := .vllmConfig | default dict -}}
{{- $deg := mul ($vc.tensorParallelSize | default 1) ($vc.pipelineParallelSize | default 1) -}}
{{- $req := .requestGPU | default 0 | int -}}
{{- if eq $req 0 -}}0{{- else -}}{{ max $req $deg }}{{- end -}}
{{- end -}}
